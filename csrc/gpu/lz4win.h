// Shared device helpers for the LZ4 decoders (ingest.hip: LDS-ring decoder, lz4seq.hip: batched
// decoder): the wave-wide compressed-stream window and an L2-coherent byte load.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zgw {

constexpr int kWave = 64;

// Compressed-stream window: three dwords per lane = bytes [wofs, wofs + 768) of the payload,
// addressed relative to the 4-byte-aligned payload base.  Reads stay inside [wofs, wofs + 320);
// the window slides by 256 bytes as the stream advances, so w2 is a 256-byte-ahead prefetch whose
// load latency overlaps parsing.  Offsets are 32-bit (a chunk payload is < 16 MiB).
struct Win {
  const uint32_t* pb;
  uint32_t wofs;
  uint32_t w0, w1, w2;
};

__device__ __forceinline__ void win_init(Win& w, const uint8_t* payload, uint32_t lane) {
  w.pb = reinterpret_cast<const uint32_t*>(payload - (reinterpret_cast<uintptr_t>(payload) & 3));
  w.wofs = 0;
  w.w0 = w.pb[lane];
  w.w1 = w.pb[kWave + lane];
  w.w2 = w.pb[2 * kWave + lane];
}

// Slide so that position a (relative to pb) is in the first 256 bytes of the window.  Callers
// advance by < 256 bytes between seeks, so at most one slide happens (an `if`, not a loop: a loop
// makes the compiler copy the freshly loaded prefetch register and wait for it immediately).
__device__ __forceinline__ void win_seek(Win& w, uint32_t a, uint32_t lane) {
  if (a >= w.wofs + 512) {  // long jump (raw block / checksum skip): reload
    w.wofs = a & ~255u;
    w.w0 = w.pb[(w.wofs >> 2) + lane];
    w.w1 = w.pb[(w.wofs >> 2) + kWave + lane];
    w.w2 = w.pb[(w.wofs >> 2) + 2 * kWave + lane];
  } else if (a >= w.wofs + 256) {
    w.wofs += 256;
    w.w0 = w.w1;
    w.w1 = w.w2;
    w.w2 = w.pb[(w.wofs >> 2) + 2 * kWave + lane];
  }
}

// Uniform byte at a (a in [wofs, wofs + 512)).
__device__ __forceinline__ uint32_t win_u8(const Win& w, uint32_t a) {
  const uint32_t rel = a - w.wofs;
  uint32_t d;
  if (rel < 256) d = __builtin_amdgcn_readlane(w.w0, int(rel >> 2));
  else d = __builtin_amdgcn_readlane(w.w1, int((rel >> 2) - 64));
  return (d >> (8 * (rel & 3))) & 0xFF;
}

// Lane i gets the byte at a + i (a in [wofs, wofs + 256)): two gathers and a select, no branch.
__device__ __forceinline__ uint32_t win_lane_u8(const Win& w, uint32_t a, uint32_t lane) {
  const uint32_t rel = a - w.wofs + lane;  // < 320: inside w0 | w1
  const uint32_t idx = (rel >> 2) & 63;
  const uint32_t d0 = __shfl(w.w0, int(idx), kWave), d1 = __shfl(w.w1, int(idx), kWave);
  return ((rel < 256 ? d0 : d1) >> (8 * (rel & 3))) & 0xFF;
}

// L2-coherent byte load (bypasses this CU's L1, which never sees its own earlier stores).
__device__ __forceinline__ uint32_t load_u8_coherent(const uint8_t* p) {
  const uint32_t k = uint32_t(reinterpret_cast<uintptr_t>(p) & 3);
  uint32_t* w = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(p - k));
  const uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (v >> (8 * k)) & 0xFF;
}

}  // namespace zgw
