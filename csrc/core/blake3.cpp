// BLAKE3 host implementation: portable compression + runtime-dispatched AVX2/AVX-512 hash_many.
#include "blake3.h"

#include <immintrin.h>

#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace zest::blake3 {

const uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                         0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

namespace {

constexpr uint8_t kMsgSchedule[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
    {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
    {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13},
};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

inline void g(uint32_t* s, int a, int b, int c, int d, uint32_t x, uint32_t y) {
  s[a] = s[a] + s[b] + x;
  s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + y;
  s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 7);
}

void compress_portable(uint32_t cv[8], const uint8_t block[64], uint8_t block_len, uint64_t counter,
                       uint8_t flags) {
  uint32_t m[16];
  for (int i = 0; i < 16; ++i) m[i] = load_le32(block + 4 * i);
  uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    kIV[0], kIV[1], kIV[2], kIV[3], uint32_t(counter), uint32_t(counter >> 32),
                    block_len, flags};
  for (int r = 0; r < 7; ++r) {
    const uint8_t* sc = kMsgSchedule[r];
    g(s, 0, 4, 8, 12, m[sc[0]], m[sc[1]]);
    g(s, 1, 5, 9, 13, m[sc[2]], m[sc[3]]);
    g(s, 2, 6, 10, 14, m[sc[4]], m[sc[5]]);
    g(s, 3, 7, 11, 15, m[sc[6]], m[sc[7]]);
    g(s, 0, 5, 10, 15, m[sc[8]], m[sc[9]]);
    g(s, 1, 6, 11, 12, m[sc[10]], m[sc[11]]);
    g(s, 2, 7, 8, 13, m[sc[12]], m[sc[13]]);
    g(s, 3, 4, 9, 14, m[sc[14]], m[sc[15]]);
  }
  for (int i = 0; i < 8; ++i) cv[i] = s[i] ^ s[i + 8];
}

void hash_many_portable(const uint8_t* const* inputs, size_t n, size_t blocks, const uint32_t key[8],
                        uint64_t counter, bool inc, uint8_t flags, uint8_t fs, uint8_t fe,
                        uint8_t* out) {
  for (size_t i = 0; i < n; ++i) {
    uint32_t cv[8];
    std::memcpy(cv, key, 32);
    const uint64_t ctr = counter + (inc ? i : 0);
    for (size_t b = 0; b < blocks; ++b) {
      uint8_t f = flags;
      if (b == 0) f |= fs;
      if (b + 1 == blocks) f |= fe;
      compress_portable(cv, inputs[i] + b * 64, 64, ctr, f);
    }
    for (int w = 0; w < 8; ++w) store_le32(out + 32 * i + 4 * w, cv[w]);
  }
}

// ------------------------------------------------------------------------------------------
// AVX2: 8 inputs in parallel, one 32-bit lane per input.
// ------------------------------------------------------------------------------------------
#define Z_AVX2 __attribute__((target("avx2")))

Z_AVX2 inline __m256i rot16_256(__m256i x) {
  const __m256i m = _mm256_setr_epi8(2, 3, 0, 1, 6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13, 2, 3, 0, 1,
                                     6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13);
  return _mm256_shuffle_epi8(x, m);
}
Z_AVX2 inline __m256i rot8_256(__m256i x) {
  const __m256i m = _mm256_setr_epi8(1, 2, 3, 0, 5, 6, 7, 4, 9, 10, 11, 8, 13, 14, 15, 12, 1, 2, 3, 0,
                                     5, 6, 7, 4, 9, 10, 11, 8, 13, 14, 15, 12);
  return _mm256_shuffle_epi8(x, m);
}
Z_AVX2 inline __m256i rot12_256(__m256i x) { return _mm256_or_si256(_mm256_srli_epi32(x, 12), _mm256_slli_epi32(x, 20)); }
Z_AVX2 inline __m256i rot7_256(__m256i x) { return _mm256_or_si256(_mm256_srli_epi32(x, 7), _mm256_slli_epi32(x, 25)); }

Z_AVX2 inline void g8(__m256i* v, int a, int b, int c, int d, __m256i x, __m256i y) {
  v[a] = _mm256_add_epi32(_mm256_add_epi32(v[a], v[b]), x);
  v[d] = rot16_256(_mm256_xor_si256(v[d], v[a]));
  v[c] = _mm256_add_epi32(v[c], v[d]);
  v[b] = rot12_256(_mm256_xor_si256(v[b], v[c]));
  v[a] = _mm256_add_epi32(_mm256_add_epi32(v[a], v[b]), y);
  v[d] = rot8_256(_mm256_xor_si256(v[d], v[a]));
  v[c] = _mm256_add_epi32(v[c], v[d]);
  v[b] = rot7_256(_mm256_xor_si256(v[b], v[c]));
}

// 8x8 transpose of 32-bit elements.
Z_AVX2 inline void transpose8(__m256i* r) {
  __m256i t0 = _mm256_unpacklo_epi32(r[0], r[1]), t1 = _mm256_unpackhi_epi32(r[0], r[1]);
  __m256i t2 = _mm256_unpacklo_epi32(r[2], r[3]), t3 = _mm256_unpackhi_epi32(r[2], r[3]);
  __m256i t4 = _mm256_unpacklo_epi32(r[4], r[5]), t5 = _mm256_unpackhi_epi32(r[4], r[5]);
  __m256i t6 = _mm256_unpacklo_epi32(r[6], r[7]), t7 = _mm256_unpackhi_epi32(r[6], r[7]);
  __m256i u0 = _mm256_unpacklo_epi64(t0, t2), u1 = _mm256_unpackhi_epi64(t0, t2);
  __m256i u2 = _mm256_unpacklo_epi64(t1, t3), u3 = _mm256_unpackhi_epi64(t1, t3);
  __m256i u4 = _mm256_unpacklo_epi64(t4, t6), u5 = _mm256_unpackhi_epi64(t4, t6);
  __m256i u6 = _mm256_unpacklo_epi64(t5, t7), u7 = _mm256_unpackhi_epi64(t5, t7);
  r[0] = _mm256_permute2x128_si256(u0, u4, 0x20);
  r[1] = _mm256_permute2x128_si256(u1, u5, 0x20);
  r[2] = _mm256_permute2x128_si256(u2, u6, 0x20);
  r[3] = _mm256_permute2x128_si256(u3, u7, 0x20);
  r[4] = _mm256_permute2x128_si256(u0, u4, 0x31);
  r[5] = _mm256_permute2x128_si256(u1, u5, 0x31);
  r[6] = _mm256_permute2x128_si256(u2, u6, 0x31);
  r[7] = _mm256_permute2x128_si256(u3, u7, 0x31);
}

Z_AVX2 void hash8_avx2(const uint8_t* const* in, size_t blocks, const uint32_t key[8], uint64_t counter,
                       bool inc, uint8_t flags, uint8_t fs, uint8_t fe, uint8_t* out) {
  __m256i h[8];
  for (int i = 0; i < 8; ++i) h[i] = _mm256_set1_epi32(int(key[i]));
  alignas(32) uint32_t clo[8], chi[8];
  for (int i = 0; i < 8; ++i) {
    uint64_t c = counter + (inc ? uint64_t(i) : 0);
    clo[i] = uint32_t(c);
    chi[i] = uint32_t(c >> 32);
  }
  const __m256i ctr_lo = _mm256_load_si256(reinterpret_cast<const __m256i*>(clo));
  const __m256i ctr_hi = _mm256_load_si256(reinterpret_cast<const __m256i*>(chi));
  for (size_t b = 0; b < blocks; ++b) {
    uint8_t f = flags;
    if (b == 0) f |= fs;
    if (b + 1 == blocks) f |= fe;
    __m256i m[16];
    for (int half = 0; half < 2; ++half) {
      __m256i* r = m + 8 * half;
      for (int i = 0; i < 8; ++i)
        r[i] = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in[i] + b * 64 + 32 * half));
      transpose8(r);
    }
    __m256i v[16] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7],
                     _mm256_set1_epi32(int(kIV[0])), _mm256_set1_epi32(int(kIV[1])),
                     _mm256_set1_epi32(int(kIV[2])), _mm256_set1_epi32(int(kIV[3])),
                     ctr_lo, ctr_hi, _mm256_set1_epi32(64), _mm256_set1_epi32(f)};
    for (int rr = 0; rr < 7; ++rr) {
      const uint8_t* sc = kMsgSchedule[rr];
      g8(v, 0, 4, 8, 12, m[sc[0]], m[sc[1]]);
      g8(v, 1, 5, 9, 13, m[sc[2]], m[sc[3]]);
      g8(v, 2, 6, 10, 14, m[sc[4]], m[sc[5]]);
      g8(v, 3, 7, 11, 15, m[sc[6]], m[sc[7]]);
      g8(v, 0, 5, 10, 15, m[sc[8]], m[sc[9]]);
      g8(v, 1, 6, 11, 12, m[sc[10]], m[sc[11]]);
      g8(v, 2, 7, 8, 13, m[sc[12]], m[sc[13]]);
      g8(v, 3, 4, 9, 14, m[sc[14]], m[sc[15]]);
    }
    for (int i = 0; i < 8; ++i) h[i] = _mm256_xor_si256(v[i], v[i + 8]);
  }
  transpose8(h);
  for (int i = 0; i < 8; ++i) _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + 32 * i), h[i]);
}

// ------------------------------------------------------------------------------------------
// AVX-512: 16 inputs in parallel.
// ------------------------------------------------------------------------------------------
#define Z_AVX512 __attribute__((target("avx512f")))

Z_AVX512 inline void g16(__m512i* v, int a, int b, int c, int d, __m512i x, __m512i y) {
  v[a] = _mm512_add_epi32(_mm512_add_epi32(v[a], v[b]), x);
  v[d] = _mm512_ror_epi32(_mm512_xor_si512(v[d], v[a]), 16);
  v[c] = _mm512_add_epi32(v[c], v[d]);
  v[b] = _mm512_ror_epi32(_mm512_xor_si512(v[b], v[c]), 12);
  v[a] = _mm512_add_epi32(_mm512_add_epi32(v[a], v[b]), y);
  v[d] = _mm512_ror_epi32(_mm512_xor_si512(v[d], v[a]), 8);
  v[c] = _mm512_add_epi32(v[c], v[d]);
  v[b] = _mm512_ror_epi32(_mm512_xor_si512(v[b], v[c]), 7);
}

// 16x16 transpose of 32-bit elements: unpack 32 -> unpack 64 -> two 128-bit-lane shuffles.
Z_AVX512 inline void transpose16(__m512i* v) {
  __m512i t[16], u[16];
  for (int i = 0; i < 8; ++i) {
    t[2 * i] = _mm512_unpacklo_epi32(v[2 * i], v[2 * i + 1]);
    t[2 * i + 1] = _mm512_unpackhi_epi32(v[2 * i], v[2 * i + 1]);
  }
  for (int i = 0; i < 4; ++i) {
    u[4 * i + 0] = _mm512_unpacklo_epi64(t[4 * i + 0], t[4 * i + 2]);
    u[4 * i + 1] = _mm512_unpackhi_epi64(t[4 * i + 0], t[4 * i + 2]);
    u[4 * i + 2] = _mm512_unpacklo_epi64(t[4 * i + 1], t[4 * i + 3]);
    u[4 * i + 3] = _mm512_unpackhi_epi64(t[4 * i + 1], t[4 * i + 3]);
  }
  for (int k = 0; k < 4; ++k) {
    __m512i w = _mm512_shuffle_i32x4(u[k], u[4 + k], 0x88);       // (2,0,2,0)
    __m512i x = _mm512_shuffle_i32x4(u[k], u[4 + k], 0xDD);       // (3,1,3,1)
    __m512i y = _mm512_shuffle_i32x4(u[8 + k], u[12 + k], 0x88);
    __m512i z = _mm512_shuffle_i32x4(u[8 + k], u[12 + k], 0xDD);
    v[0 + k] = _mm512_shuffle_i32x4(w, y, 0x88);
    v[8 + k] = _mm512_shuffle_i32x4(w, y, 0xDD);
    v[4 + k] = _mm512_shuffle_i32x4(x, z, 0x88);
    v[12 + k] = _mm512_shuffle_i32x4(x, z, 0xDD);
  }
}

Z_AVX512 void hash16_avx512(const uint8_t* const* in, size_t blocks, const uint32_t key[8],
                            uint64_t counter, bool inc, uint8_t flags, uint8_t fs, uint8_t fe,
                            uint8_t* out) {
  __m512i h[8];
  for (int i = 0; i < 8; ++i) h[i] = _mm512_set1_epi32(int(key[i]));
  alignas(64) uint32_t clo[16], chi[16];
  for (int i = 0; i < 16; ++i) {
    uint64_t c = counter + (inc ? uint64_t(i) : 0);
    clo[i] = uint32_t(c);
    chi[i] = uint32_t(c >> 32);
  }
  const __m512i ctr_lo = _mm512_load_si512(clo);
  const __m512i ctr_hi = _mm512_load_si512(chi);
  for (size_t b = 0; b < blocks; ++b) {
    uint8_t f = flags;
    if (b == 0) f |= fs;
    if (b + 1 == blocks) f |= fe;
    __m512i m[16];
    for (int i = 0; i < 16; ++i) m[i] = _mm512_loadu_si512(in[i] + b * 64);
    transpose16(m);
    __m512i v[16] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7],
                     _mm512_set1_epi32(int(kIV[0])), _mm512_set1_epi32(int(kIV[1])),
                     _mm512_set1_epi32(int(kIV[2])), _mm512_set1_epi32(int(kIV[3])),
                     ctr_lo, ctr_hi, _mm512_set1_epi32(64), _mm512_set1_epi32(f)};
    for (int rr = 0; rr < 7; ++rr) {
      const uint8_t* sc = kMsgSchedule[rr];
      g16(v, 0, 4, 8, 12, m[sc[0]], m[sc[1]]);
      g16(v, 1, 5, 9, 13, m[sc[2]], m[sc[3]]);
      g16(v, 2, 6, 10, 14, m[sc[4]], m[sc[5]]);
      g16(v, 3, 7, 11, 15, m[sc[6]], m[sc[7]]);
      g16(v, 0, 5, 10, 15, m[sc[8]], m[sc[9]]);
      g16(v, 1, 6, 11, 12, m[sc[10]], m[sc[11]]);
      g16(v, 2, 7, 8, 13, m[sc[12]], m[sc[13]]);
      g16(v, 3, 4, 9, 14, m[sc[14]], m[sc[15]]);
    }
    for (int i = 0; i < 8; ++i) h[i] = _mm512_xor_si512(v[i], v[i + 8]);
  }
  // h[w] lane i = word w of input i.  Write out per input.
  alignas(64) uint32_t tmp[8][16];
  for (int w = 0; w < 8; ++w) _mm512_store_si512(tmp[w], h[w]);
  for (int i = 0; i < 16; ++i)
    for (int w = 0; w < 8; ++w) store_le32(out + 32 * i + 4 * w, tmp[w][i]);
}

enum class Backend { Portable, Avx2, Avx512 };

Backend detect() {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f")) return Backend::Avx512;
  if (__builtin_cpu_supports("avx2")) return Backend::Avx2;
  return Backend::Portable;
}

Backend g_backend = detect();

// One chunk (<= 1024 bytes) -> output node {cv, block, block_len, counter, flags} so the caller
// can finalize as ROOT or take the chaining value.
struct OutputNode {
  uint32_t cv[8];
  uint8_t block[64];
  uint8_t block_len;
  uint64_t counter;
  uint8_t flags;
};

OutputNode chunk_output(const uint32_t key[8], uint8_t flags, const uint8_t* data, size_t len,
                        uint64_t counter) {
  OutputNode o;
  std::memcpy(o.cv, key, 32);
  size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b + 1 < nblocks; ++b) {
    uint8_t f = flags | (b == 0 ? CHUNK_START : 0);
    compress_portable(o.cv, data + 64 * b, 64, counter, f);
  }
  size_t last = (nblocks - 1) * 64;
  size_t last_len = len - last;
  std::memset(o.block, 0, 64);
  if (last_len) std::memcpy(o.block, data + last, last_len);
  o.block_len = uint8_t(last_len);
  o.counter = counter;
  o.flags = flags | CHUNK_END | (nblocks == 1 ? CHUNK_START : 0);
  return o;
}

void output_root(const OutputNode& o, uint8_t out[32]) {
  uint32_t cv[8];
  std::memcpy(cv, o.cv, 32);
  compress_portable(cv, o.block, o.block_len, 0, o.flags | ROOT);
  for (int w = 0; w < 8; ++w) store_le32(out + 4 * w, cv[w]);
}

void output_cv(const OutputNode& o, uint8_t out[32]) {
  uint32_t cv[8];
  std::memcpy(cv, o.cv, 32);
  compress_portable(cv, o.block, o.block_len, o.counter, o.flags);
  for (int w = 0; w < 8; ++w) store_le32(out + 4 * w, cv[w]);
}

}  // namespace

void compress_in_place(uint32_t cv[8], const uint8_t block[64], uint8_t block_len, uint64_t counter,
                       uint8_t flags) {
  compress_portable(cv, block, block_len, counter, flags);
}

void hash_many(const uint8_t* const* inputs, size_t n, size_t blocks, const uint32_t key[8],
               uint64_t counter, bool inc, uint8_t flags, uint8_t fs, uint8_t fe, uint8_t* out) {
  size_t i = 0;
  if (g_backend == Backend::Avx512) {
    for (; i + 16 <= n; i += 16)
      hash16_avx512(inputs + i, blocks, key, counter + (inc ? i : 0), inc, flags, fs, fe, out + 32 * i);
  }
  if (g_backend != Backend::Portable) {
    for (; i + 8 <= n; i += 8)
      hash8_avx2(inputs + i, blocks, key, counter + (inc ? i : 0), inc, flags, fs, fe, out + 32 * i);
  }
  if (i < n)
    hash_many_portable(inputs + i, n - i, blocks, key, counter + (inc ? i : 0), inc, flags, fs, fe,
                       out + 32 * i);
}

void hash_with_key(const uint32_t key[8], uint8_t flags, const void* vdata, size_t len, uint8_t out[32]) {
  const uint8_t* data = static_cast<const uint8_t*>(vdata);
  if (len <= kChunkLen) {
    output_root(chunk_output(key, flags, data, len, 0), out);
    return;
  }
  const size_t n_chunks = (len + kChunkLen - 1) / kChunkLen;
  const size_t n_full = len / kChunkLen;  // complete 1 KiB chunks (the last may be full too)
  uint8_t stack_cvs[64 * 32];
  std::vector<uint8_t> heap_cvs;
  uint8_t* cvs = stack_cvs;
  if (n_chunks > 64) {
    heap_cvs.resize(n_chunks * 32);
    cvs = heap_cvs.data();
  }
  {
    const uint8_t* ptrs[16];
    size_t c = 0;
    while (c < n_full) {
      size_t k = std::min<size_t>(16, n_full - c);
      for (size_t j = 0; j < k; ++j) ptrs[j] = data + (c + j) * kChunkLen;
      hash_many(ptrs, k, kChunkLen / kBlockLen, key, c, true, flags, CHUNK_START, CHUNK_END, cvs + 32 * c);
      c += k;
    }
    if (n_full < n_chunks) {
      const size_t off = n_full * kChunkLen;
      output_cv(chunk_output(key, flags, data + off, len - off, n_full), cvs + 32 * n_full);
    }
  }
  // Pairwise merge with carry == BLAKE3's left-complete tree.
  size_t count = n_chunks;
  while (count > 2) {
    const size_t pairs = count / 2;
    const uint8_t* ptrs[16];
    size_t p = 0;
    std::vector<uint8_t> tmp(pairs * 32);
    while (p < pairs) {
      size_t k = std::min<size_t>(16, pairs - p);
      for (size_t j = 0; j < k; ++j) ptrs[j] = cvs + 64 * (p + j);
      hash_many(ptrs, k, 1, key, 0, false, flags | PARENT, 0, 0, tmp.data() + 32 * p);
      p += k;
    }
    std::memcpy(cvs, tmp.data(), pairs * 32);
    if (count & 1) std::memmove(cvs + 32 * pairs, cvs + 32 * (count - 1), 32);
    count = pairs + (count & 1);
  }
  uint32_t cv[8];
  std::memcpy(cv, key, 32);
  compress_portable(cv, cvs, 64, 0, flags | PARENT | ROOT);
  for (int w = 0; w < 8; ++w) store_le32(out + 4 * w, cv[w]);
}

void hash(const void* data, size_t len, uint8_t out[32]) { hash_with_key(kIV, 0, data, len, out); }

void keyed_hash(const uint8_t key[32], const void* data, size_t len, uint8_t out[32]) {
  uint32_t kw[8];
  for (int i = 0; i < 8; ++i) kw[i] = load_le32(key + 4 * i);
  hash_with_key(kw, KEYED_HASH, data, len, out);
}

const char* simd_backend() {
  switch (g_backend) {
    case Backend::Avx512: return "avx512";
    case Backend::Avx2: return "avx2";
    default: return "portable";
  }
}

bool force_backend(const char* name) {
  std::string n(name);
  Backend best = detect();
  if (n == "portable") { g_backend = Backend::Portable; return true; }
  if (n == "avx2" && best != Backend::Portable) { g_backend = Backend::Avx2; return true; }
  if (n == "avx512" && best == Backend::Avx512) { g_backend = Backend::Avx512; return true; }
  if (n == "auto") { g_backend = best; return true; }
  return false;
}

}  // namespace zest::blake3
