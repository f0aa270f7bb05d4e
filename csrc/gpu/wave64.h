// Wave64 cross-lane primitives for gfx950 (CDNA4): DPP inclusive scans.
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

}  // namespace zwv
