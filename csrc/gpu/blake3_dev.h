// Device BLAKE3 for CDNA4 (gfx950): compression fully unrolled in VGPRs, rotations as
// v_alignbit_b32, a+b+m as v_add3_u32.  One lane owns one 1 KiB BLAKE3 chunk (16 chained
// compressions); parents are merged across lanes through LDS (see ingest.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zg {

constexpr uint32_t kIV0 = 0x6A09E667u, kIV1 = 0xBB67AE85u, kIV2 = 0x3C6EF372u, kIV3 = 0xA54FF53Au,
                   kIV4 = 0x510E527Fu, kIV5 = 0x9B05688Cu, kIV6 = 0x1F83D9ABu, kIV7 = 0x5BE0CD19u;
constexpr uint32_t CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8, KEYED_HASH = 16;

// Key words (little-endian) of the Xet keys.
struct Key8 {
  uint32_t w[8];
};
__device__ __constant__ static const Key8 kDataKeyW = {{0x77f59766u, 0xde50955bu, 0xaccb3531u, 0x1c1897a5u,
                                                        0x1021e49du, 0x582beb9bu, 0x4bb0d0b4u, 0x29f2ad93u}};
__device__ __constant__ static const Key8 kNodeKeyW = {{0xc7c57e01u, 0x962947a5u, 0x666694fdu, 0xe6028ab4u,
                                                        0x6f53dd5du, 0xd26dc737u, 0xe65263f8u, 0x3f71534au}};
__device__ __constant__ static const Key8 kIVW = {{kIV0, kIV1, kIV2, kIV3, kIV4, kIV5, kIV6, kIV7}};
__device__ __constant__ static const Key8 kZeroW = {{0, 0, 0, 0, 0, 0, 0, 0}};

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }

#define ZG_G(a, b, c, d, x, y) \
  a = a + b + (x);             \
  d = rotr(d ^ a, 16);         \
  c = c + d;                   \
  b = rotr(b ^ c, 12);         \
  a = a + b + (y);             \
  d = rotr(d ^ a, 8);          \
  c = c + d;                   \
  b = rotr(b ^ c, 7);

#define ZG_ROUND(m)                                   \
  ZG_G(v0, v4, v8, v12, m[0], m[1]);                 \
  ZG_G(v1, v5, v9, v13, m[2], m[3]);                 \
  ZG_G(v2, v6, v10, v14, m[4], m[5]);                \
  ZG_G(v3, v7, v11, v15, m[6], m[7]);                \
  ZG_G(v0, v5, v10, v15, m[8], m[9]);                \
  ZG_G(v1, v6, v11, v12, m[10], m[11]);              \
  ZG_G(v2, v7, v8, v13, m[12], m[13]);               \
  ZG_G(v3, v4, v9, v14, m[14], m[15]);

// Message permutation between rounds: m'[i] = m[P[i]], P = {2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8}.
#define ZG_PERMUTE(m)                                                                      \
  {                                                                                        \
    uint32_t t0 = m[0], t1 = m[1], t2 = m[2], t3 = m[3], t4 = m[4], t5 = m[5], t6 = m[6], \
             t7 = m[7], t8 = m[8], t9 = m[9], t10 = m[10], t11 = m[11], t12 = m[12],       \
             t13 = m[13], t14 = m[14], t15 = m[15];                                        \
    m[0] = t2; m[1] = t6; m[2] = t3; m[3] = t10; m[4] = t7; m[5] = t0; m[6] = t4;          \
    m[7] = t13; m[8] = t1; m[9] = t11; m[10] = t12; m[11] = t5; m[12] = t9; m[13] = t14;   \
    m[14] = t15; m[15] = t8;                                                               \
  }

// cv <- compress(cv, m, counter, block_len, flags)[0..8]
__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t min[16], uint64_t counter,
                                         uint32_t block_len, uint32_t flags) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = min[i];
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
  uint32_t v8 = kIV0, v9 = kIV1, v10 = kIV2, v11 = kIV3;
  uint32_t v12 = uint32_t(counter), v13 = uint32_t(counter >> 32), v14 = block_len, v15 = flags;
  ZG_ROUND(m) ZG_PERMUTE(m)
  ZG_ROUND(m) ZG_PERMUTE(m)
  ZG_ROUND(m) ZG_PERMUTE(m)
  ZG_ROUND(m) ZG_PERMUTE(m)
  ZG_ROUND(m) ZG_PERMUTE(m)
  ZG_ROUND(m) ZG_PERMUTE(m)
  ZG_ROUND(m)
  cv[0] = v0 ^ v8;
  cv[1] = v1 ^ v9;
  cv[2] = v2 ^ v10;
  cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12;
  cv[5] = v5 ^ v13;
  cv[6] = v6 ^ v14;
  cv[7] = v7 ^ v15;
}

__device__ __forceinline__ void load_key(uint32_t cv[8], const Key8& k) {
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = k.w[i];
}

// Load 64 bytes starting at an arbitrary byte address into 16 little-endian words, zeroing
// bytes at or beyond `avail` (0..64).  Reads whole aligned dwords; the caller guarantees the
// buffer is padded so that the covering aligned dwords are readable.
__device__ __forceinline__ void load_block(const uint8_t* p, uint32_t avail, uint32_t m[16]) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t k = uint32_t(a & 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  if (k == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = w[i];
  } else {
    uint32_t prev = w[0];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t nxt = w[i + 1];
      m[i] = __builtin_amdgcn_alignbyte(nxt, prev, k);
      prev = nxt;
    }
  }
  if (avail < 64) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int lo = 4 * i;
      uint32_t keep;
      if (int(avail) >= lo + 4) keep = 0xFFFFFFFFu;
      else if (int(avail) <= lo) keep = 0u;
      else keep = 0xFFFFFFFFu >> (8 * (lo + 4 - int(avail)));
      m[i] &= keep;
    }
  }
}

// Hash one <= 1 KiB BLAKE3 chunk starting at p (len bytes) with counter `chunk_idx`.
// If `is_root` (the whole message is this single chunk), the final block gets ROOT and the
// returned cv is the hash.
__device__ __forceinline__ void hash_chunk(const uint8_t* p, uint32_t len, uint64_t chunk_idx,
                                           const Key8& key, uint32_t mode_flags, bool is_root,
                                           uint32_t cv[8]) {
  load_key(cv, key);
  const uint32_t nblk = len == 0 ? 1 : (len + 63) / 64;
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t m[16];
    const uint32_t avail = len - 64 * b < 64 ? len - 64 * b : 64;
    if (len == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = 0;
    } else {
      load_block(p + 64 * b, avail, m);
    }
    uint32_t f = mode_flags;
    if (b == 0) f |= CHUNK_START;
    if (b + 1 == nblk) {
      f |= CHUNK_END;
      if (is_root) f |= ROOT;
    }
    compress(cv, m, is_root ? 0 : chunk_idx, avail, f);
  }
}

// 17 consecutive dwords from a 4-byte-aligned address (the 64-byte block plus the next dword that
// the byte-alignment shift needs): four 16-byte loads + one dword.
// (global address space, so they issue as global_load and not flat_load, which would also count
// against lgkmcnt and serialize with the LDS/scalar waits)
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const __attribute__((address_space(1))) u32x4_a4* gq4_t;
typedef const __attribute__((address_space(1))) uint32_t* gw_t;
__device__ __forceinline__ void fetch17(const uint32_t* w, uint32_t r[17]) {
  gq4_t q = (gq4_t)w;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4_a4 v = q[i];
    r[4 * i] = v.x;
    r[4 * i + 1] = v.y;
    r[4 * i + 2] = v.z;
    r[4 * i + 3] = v.w;
  }
  r[16] = ((gw_t)w)[16];
}

// One <= 1 KiB BLAKE3 chunk like hash_chunk, with block b+1's loads in flight while block b
// compresses (the lane's 1 KiB is read as 16 x 64 B; a shift of k bytes realigns every word with
// v_alignbyte, which is the identity for k == 0, so there is no aligned/unaligned branch).
__device__ __forceinline__ void hash_leaf(const uint8_t* p, uint32_t len, uint64_t counter, const Key8& key,
                                          uint32_t mode_flags, bool is_root, uint32_t cv[8]) {
  load_key(cv, key);
  const uint32_t nblk = len == 0 ? 1 : (len + 63) >> 6;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t k = uint32_t(a & 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  uint32_t cur[17];
  if (len) {
    fetch17(w, cur);
  } else {
#pragma unroll
    for (int i = 0; i < 17; ++i) cur[i] = 0;
  }
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t nxt[17];
    if (b + 1 < nblk) fetch17(w + 16 * (b + 1), nxt);
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = __builtin_amdgcn_alignbyte(cur[i + 1], cur[i], k);
    const uint32_t avail = len - 64 * b < 64 ? len - 64 * b : 64;
    if (avail < 64) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int lo = 4 * i;
        uint32_t keep;
        if (int(avail) >= lo + 4) keep = 0xFFFFFFFFu;
        else if (int(avail) <= lo) keep = 0u;
        else keep = 0xFFFFFFFFu >> (8 * (lo + 4 - int(avail)));
        m[i] &= keep;
      }
    }
    uint32_t f = mode_flags;
    if (b == 0) f |= CHUNK_START;
    if (b + 1 == nblk) f |= CHUNK_END | (is_root ? ROOT : 0u);
    compress(cv, m, is_root ? 0 : counter, avail, f);
#pragma unroll
    for (int i = 0; i < 17; ++i) cur[i] = nxt[i];
  }
}

__device__ __forceinline__ void parent_cv(const uint32_t l[8], const uint32_t r[8], const Key8& key,
                                          uint32_t mode_flags, bool root, uint32_t out[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = l[i];
    m[8 + i] = r[i];
  }
  load_key(out, key);
  compress(out, m, 0, 64, mode_flags | PARENT | (root ? ROOT : 0));
}

// One wave hashes one Xet chunk (<= 128 KiB): lane l owns BLAKE3 chunks l, l + 64; chaining values
// are merged pairwise in `cvs` (LDS, 8 words per BLAKE3 chunk, 4 KiB for 128 of them) --
// pairwise-with-carry is BLAKE3's left-complete tree.  K1's latency path (k_hash_chunks) and the
// fused hash at the end of the LZ4 pair decoder (lz4seq.hip).
__device__ inline void wave_hash(const uint8_t* base, uint32_t len, const Key8& key, uint32_t mode, uint32_t* cvs,
                          uint32_t lane, uint32_t out[8]) {
  const uint32_t nb = len == 0 ? 1 : (len + 1023) >> 10;
  if (nb == 1) {
    uint32_t cv[8];
    if (lane == 0) hash_chunk(base, len, 0, key, mode, true, cv);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = __builtin_amdgcn_readfirstlane(cv[i]);
    return;
  }
  for (uint32_t b = lane; b < nb; b += 64) {
    const uint32_t seg = len - (b << 10) < 1024 ? len - (b << 10) : 1024;
    uint32_t cv[8];
    hash_chunk(base + (size_t(b) << 10), seg, b, key, mode, false, cv);
#pragma unroll
    for (int i = 0; i < 8; ++i) cvs[8 * b + i] = cv[i];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t m = nb;
  while (m > 2) {
    const uint32_t pairs = m >> 1;
    for (uint32_t i = lane; i < pairs; i += 64) {
      uint32_t l[8], r[8], o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        l[k] = cvs[16 * i + k];
        r[k] = cvs[16 * i + 8 + k];
      }
      parent_cv(l, r, key, mode, false, o);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 8; ++k) cvs[8 * i + k] = o[k];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (m & 1) {
      if (lane < 8) cvs[8 * pairs + lane] = cvs[8 * (m - 1) + lane];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    m = pairs + (m & 1);
  }
  uint32_t l[8], r[8], o[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    l[k] = cvs[k];
    r[k] = cvs[8 + k];
  }
  parent_cv(l, r, key, mode, true, o);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = o[k];
}

__device__ __forceinline__ void store_hash(uint8_t* dst, const uint32_t h[8], uint32_t lane) {
  if (lane < 8) reinterpret_cast<uint32_t*>(dst)[lane] = h[0] * (lane == 0) + h[1] * (lane == 1) + h[2] * (lane == 2) +
                                                          h[3] * (lane == 3) + h[4] * (lane == 4) + h[5] * (lane == 5) +
                                                          h[6] * (lane == 6) + h[7] * (lane == 7);
}

}  // namespace zg
