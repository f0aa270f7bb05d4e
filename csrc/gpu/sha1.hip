// K6: batch SHA-1 info-hashes on the GPU — SHA1("zest-xet-v1:" || xorb_hash) for many xorbs at
// once (one BitTorrent swarm per xorb, reference src/peer_id.zig:21-33).  44-byte messages are one
// SHA-1 block after padding, so each thread runs exactly one 80-round compression with its message
// schedule in a 16-word rolling window (registers only).  Host twin: csrc/core/sha1.cpp.
#include <hip/hip_runtime.h>

#include "zgpu.h"

namespace {

__device__ __forceinline__ uint32_t rol(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__global__ void __launch_bounds__(256) k_sha1_info_hash(const uint8_t* __restrict__ hashes, int n,
                                                        uint8_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // message words (big-endian): "zest" "-xet" "-v1:" then 8 words of the hash, 0x80 pad, length 352
  const uint32_t* h = reinterpret_cast<const uint32_t*>(hashes + 32 * size_t(i));
  uint32_t w[16];
  w[0] = 0x7a657374u;  // "zest"
  w[1] = 0x2d786574u;  // "-xet"
  w[2] = 0x2d76313au;  // "-v1:"
#pragma unroll
  for (int k = 0; k < 8; ++k) w[3 + k] = bswap(h[k]);
  w[11] = 0x80000000u;
  w[12] = w[13] = w[14] = 0;
  w[15] = 44 * 8;
  uint32_t a = 0x67452301u, b = 0xEFCDAB89u, c = 0x98BADCFEu, d = 0x10325476u, e = 0xC3D2E1F0u;
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      wt = rol(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
      w[t & 15] = wt;
    }
    uint32_t f, k;
    if (t < 20) {
      f = (b & c) | (~b & d);
      k = 0x5A827999u;
    } else if (t < 40) {
      f = b ^ c ^ d;
      k = 0x6ED9EBA1u;
    } else if (t < 60) {
      f = (b & c) | (b & d) | (c & d);
      k = 0x8F1BBCDCu;
    } else {
      f = b ^ c ^ d;
      k = 0xCA62C1D6u;
    }
    const uint32_t tmp = rol(a, 5) + f + e + k + wt;
    e = d;
    d = c;
    c = rol(b, 30);
    b = a;
    a = tmp;
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(out + 20 * size_t(i));
  o[0] = bswap(a + 0x67452301u);
  o[1] = bswap(b + 0xEFCDAB89u);
  o[2] = bswap(c + 0x98BADCFEu);
  o[3] = bswap(d + 0x10325476u);
  o[4] = bswap(e + 0xC3D2E1F0u);
}

}  // namespace

extern "C" hipError_t zg_sha1_info_hash(const uint8_t* hashes, int n, uint8_t* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha1_info_hash, dim3((n + 255) / 256), dim3(256), 0, stream, hashes, n, out);
  return hipGetLastError();
}
