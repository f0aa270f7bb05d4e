#include "sha1.h"

#include <immintrin.h>

#include <cstring>
#include <random>

#include "common.h"

namespace zest {

namespace {

inline uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

void block_portable(uint32_t h[5], const uint8_t* p, size_t nblocks) {
  for (size_t b = 0; b < nblocks; ++b, p += 64) {
    uint32_t w[80];
    for (int i = 0; i < 16; ++i) w[i] = load_be32(p + 4 * i);
    for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; ++i) {
      uint32_t f, k;
      if (i < 20) {
        f = (bb & c) | (~bb & d);
        k = 0x5A827999u;
      } else if (i < 40) {
        f = bb ^ c ^ d;
        k = 0x6ED9EBA1u;
      } else if (i < 60) {
        f = (bb & c) | (bb & d) | (c & d);
        k = 0x8F1BBCDCu;
      } else {
        f = bb ^ c ^ d;
        k = 0xCA62C1D6u;
      }
      const uint32_t t = rol(a, 5) + f + e + k + w[i];
      e = d;
      d = c;
      c = rol(bb, 30);
      bb = a;
      a = t;
    }
    h[0] += a;
    h[1] += bb;
    h[2] += c;
    h[3] += d;
    h[4] += e;
  }
}

#define Z_SHA __attribute__((target("sha,sse4.1,ssse3")))

Z_SHA void block_shani(uint32_t state[5], const uint8_t* data, size_t nblocks) {
  const __m128i MASK = _mm_set_epi64x(0x0001020304050607ULL, 0x08090a0b0c0d0e0fULL);
  __m128i ABCD = _mm_loadu_si128(reinterpret_cast<const __m128i*>(state));
  __m128i E0 = _mm_set_epi32(int(state[4]), 0, 0, 0);
  ABCD = _mm_shuffle_epi32(ABCD, 0x1B);
  __m128i E1, MSG0, MSG1, MSG2, MSG3;
  while (nblocks--) {
    const __m128i ABCD_SAVE = ABCD, E0_SAVE = E0;
#define LD(o) _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + (o))), MASK)
    MSG0 = LD(0);
    E0 = _mm_add_epi32(E0, MSG0);
    E1 = ABCD;
    ABCD = _mm_sha1rnds4_epu32(ABCD, E0, 0);
    MSG1 = LD(16);
    E1 = _mm_sha1nexte_epu32(E1, MSG1);
    E0 = ABCD;
    ABCD = _mm_sha1rnds4_epu32(ABCD, E1, 0);
    MSG0 = _mm_sha1msg1_epu32(MSG0, MSG1);
    MSG2 = LD(32);
    E0 = _mm_sha1nexte_epu32(E0, MSG2);
    E1 = ABCD;
    ABCD = _mm_sha1rnds4_epu32(ABCD, E0, 0);
    MSG1 = _mm_sha1msg1_epu32(MSG1, MSG2);
    MSG0 = _mm_xor_si128(MSG0, MSG2);
    MSG3 = LD(48);
#undef LD
    // Rounds 12..67: the standard 4-message rotation.
#define R4(EA, EB, MA, MB, MC, MD, F)            \
  EA = _mm_sha1nexte_epu32(EA, MA);              \
  EB = ABCD;                                     \
  MB = _mm_sha1msg2_epu32(MB, MA);               \
  ABCD = _mm_sha1rnds4_epu32(ABCD, EA, F);       \
  MD = _mm_sha1msg1_epu32(MD, MA);               \
  MC = _mm_xor_si128(MC, MA);
    // rounds 12-15 (nexte with MSG3; msg2 into MSG0)
    E1 = _mm_sha1nexte_epu32(E1, MSG3);
    E0 = ABCD;
    MSG0 = _mm_sha1msg2_epu32(MSG0, MSG3);
    ABCD = _mm_sha1rnds4_epu32(ABCD, E1, 0);
    MSG2 = _mm_sha1msg1_epu32(MSG2, MSG3);
    MSG1 = _mm_xor_si128(MSG1, MSG3);
    R4(E0, E1, MSG0, MSG1, MSG2, MSG3, 0)  // 16-19
    R4(E1, E0, MSG1, MSG2, MSG3, MSG0, 1)  // 20-23
    R4(E0, E1, MSG2, MSG3, MSG0, MSG1, 1)  // 24-27
    R4(E1, E0, MSG3, MSG0, MSG1, MSG2, 1)  // 28-31
    R4(E0, E1, MSG0, MSG1, MSG2, MSG3, 1)  // 32-35
    R4(E1, E0, MSG1, MSG2, MSG3, MSG0, 1)  // 36-39
    R4(E0, E1, MSG2, MSG3, MSG0, MSG1, 2)  // 40-43
    R4(E1, E0, MSG3, MSG0, MSG1, MSG2, 2)  // 44-47
    R4(E0, E1, MSG0, MSG1, MSG2, MSG3, 2)  // 48-51
    R4(E1, E0, MSG1, MSG2, MSG3, MSG0, 2)  // 52-55
    R4(E0, E1, MSG2, MSG3, MSG0, MSG1, 2)  // 56-59
    R4(E1, E0, MSG3, MSG0, MSG1, MSG2, 3)  // 60-63
    R4(E0, E1, MSG0, MSG1, MSG2, MSG3, 3)  // 64-67
#undef R4
    // 68-71
    E1 = _mm_sha1nexte_epu32(E1, MSG1);
    E0 = ABCD;
    MSG2 = _mm_sha1msg2_epu32(MSG2, MSG1);
    ABCD = _mm_sha1rnds4_epu32(ABCD, E1, 3);
    MSG3 = _mm_xor_si128(MSG3, MSG1);
    // 72-75
    E0 = _mm_sha1nexte_epu32(E0, MSG2);
    E1 = ABCD;
    MSG3 = _mm_sha1msg2_epu32(MSG3, MSG2);
    ABCD = _mm_sha1rnds4_epu32(ABCD, E0, 3);
    // 76-79
    E1 = _mm_sha1nexte_epu32(E1, MSG3);
    E0 = ABCD;
    ABCD = _mm_sha1rnds4_epu32(ABCD, E1, 3);
    E0 = _mm_sha1nexte_epu32(E0, E0_SAVE);
    ABCD = _mm_add_epi32(ABCD, ABCD_SAVE);
    data += 64;
  }
  ABCD = _mm_shuffle_epi32(ABCD, 0x1B);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(state), ABCD);
  state[4] = uint32_t(_mm_extract_epi32(E0, 3));
}

bool detect_shani() {
  __builtin_cpu_init();
  unsigned a, b, c, d;
  if (!__builtin_cpu_supports("ssse3") || !__builtin_cpu_supports("sse4.1")) return false;
  __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
  return (b >> 29) & 1;  // CPUID.(EAX=7,ECX=0):EBX.SHA[bit 29]
}

const bool g_shani = detect_shani();

inline void blocks(uint32_t h[5], const uint8_t* p, size_t n) {
  if (g_shani) block_shani(h, p, n);
  else block_portable(h, p, n);
}

}  // namespace

Sha1::Sha1() : h_{0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u} {}

void Sha1::update(const void* vdata, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(vdata);
  total_ += n;
  if (buf_len_) {
    size_t take = std::min(n, 64 - buf_len_);
    std::memcpy(buf_ + buf_len_, p, take);
    buf_len_ += take;
    p += take;
    n -= take;
    if (buf_len_ == 64) {
      blocks(h_, buf_, 1);
      buf_len_ = 0;
    }
  }
  if (n >= 64) {
    blocks(h_, p, n / 64);
    p += n / 64 * 64;
    n %= 64;
  }
  if (n) {
    std::memcpy(buf_, p, n);
    buf_len_ = n;
  }
}

Sha1Digest Sha1::finish() {
  uint8_t pad[128] = {0};
  const size_t len = buf_len_;
  std::memcpy(pad, buf_, len);
  pad[len] = 0x80;
  const size_t total_len = len + 1 + 8 <= 64 ? 64 : 128;
  const uint64_t bits = total_ * 8;
  for (int i = 0; i < 8; ++i) pad[total_len - 1 - i] = uint8_t(bits >> (8 * i));
  blocks(h_, pad, total_len / 64);
  Sha1Digest d;
  for (int i = 0; i < 5; ++i) store_be32(d.data() + 4 * i, h_[i]);
  return d;
}

Sha1Digest Sha1::hash(const void* data, size_t n) {
  Sha1 s;
  s.update(data, n);
  return s.finish();
}

const char* Sha1::backend() { return g_shani ? "sha-ni" : "portable"; }

namespace peer_id {

PeerId generate() {
  PeerId id;
  std::memcpy(id.data(), kClientPrefix, 8);
  std::random_device rd;
  for (int i = 8; i < 20; ++i) id[i] = uint8_t(rd());
  return id;
}

Sha1Digest info_hash(const uint8_t xorb_hash[32]) {
  // 12-byte prefix + 32-byte hash = 44 bytes: exactly one SHA-1 block after padding.
  uint8_t block[64] = {0};
  std::memcpy(block, kInfoHashPrefix, 12);
  std::memcpy(block + 12, xorb_hash, 32);
  block[44] = 0x80;
  block[62] = uint8_t((44 * 8) >> 8);
  block[63] = uint8_t(44 * 8);
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  blocks(h, block, 1);
  Sha1Digest d;
  for (int i = 0; i < 5; ++i) store_be32(d.data() + 4 * i, h[i]);
  return d;
}

}  // namespace peer_id

}  // namespace zest
