// Wave64 cross-lane primitives for gfx950 (CDNA4): DPP inclusive scans, wave-cooperative copy.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zwv {

// row_shr:1/2/4/8 within 16-lane rows, then row_bcast:15 / row_bcast:31 across rows (gfx9 DPP):
// six VALU ops per scan instead of six LDS permutes.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), kCtrl, kRowMask, 0xF, false));
}
__device__ __forceinline__ uint32_t scan_add(uint32_t v) {
  v += dpp<0x111, 0xF>(v);
  v += dpp<0x112, 0xF>(v);
  v += dpp<0x114, 0xF>(v);
  v += dpp<0x118, 0xF>(v);
  v += dpp<0x142, 0xA>(v);
  v += dpp<0x143, 0xC>(v);
  return v;
}
__device__ __forceinline__ uint32_t scan_max(uint32_t v) {
  v = max(v, dpp<0x111, 0xF>(v));
  v = max(v, dpp<0x112, 0xF>(v));
  v = max(v, dpp<0x114, 0xF>(v));
  v = max(v, dpp<0x118, 0xF>(v));
  v = max(v, dpp<0x142, 0xA>(v));
  v = max(v, dpp<0x143, 0xC>(v));
  return v;
}

// --------------------------------------------------------------------------------------------
// Wave-cooperative byte-exact copy between arbitrarily aligned addresses: 16-byte aligned
// dwordx4 stores; the source is read as aligned dwords and funnel-shifted (v_alignbyte_b32).
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_copy(uint8_t* d, const uint8_t* s, uint64_t n, uint32_t lane) {
  constexpr int kWave = 64;
  const uint64_t da = reinterpret_cast<uintptr_t>(d);
  uint64_t head = (16 - (da & 15)) & 15;
  if (head > n) head = n;
  if (lane < head) d[lane] = s[lane];
  d += head;
  s += head;
  n -= head;
  const uint64_t nvec = n >> 4;
  const uintptr_t sa = reinterpret_cast<uintptr_t>(s);
  const uint32_t k = uint32_t(sa & 3);
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(sa & ~uintptr_t(3));
  uint4* dv = reinterpret_cast<uint4*>(d);
  if (k == 0) {
    for (uint64_t v = lane; v < nvec; v += kWave) {
      const uint32_t* p = sw + 4 * v;
      uint4 o;
      o.x = p[0];
      o.y = p[1];
      o.z = p[2];
      o.w = p[3];
      dv[v] = o;
    }
  } else {
    for (uint64_t v = lane; v < nvec; v += kWave) {
      const uint32_t* p = sw + 4 * v;
      const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
      uint4 o;
      o.x = __builtin_amdgcn_alignbyte(w1, w0, k);
      o.y = __builtin_amdgcn_alignbyte(w2, w1, k);
      o.z = __builtin_amdgcn_alignbyte(w3, w2, k);
      o.w = __builtin_amdgcn_alignbyte(w4, w3, k);
      dv[v] = o;
    }
  }
  const uint64_t done = nvec << 4;
  const uint64_t rem = n - done;
  if (lane < rem) d[done + lane] = s[done + lane];
}

}  // namespace zwv
