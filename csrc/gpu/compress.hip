// K7b: Xet chunk compression on MI355X (gfx950): BG4 byte grouping + LZ4 frame, one wave per chunk.
// SURVEY §2.G K7 ("xorb assembly, optionally compress").  Output frames use the same layout as the
// host encoder (csrc/core/lz4.cpp::compress_frame: FLG 0x60, one independent block, no checksums), so
// the host decoder, hf_xet and k_decode_lz4 all read them.
//
// Match finding is window-parallel: the 64 lanes look up positions ip .. ip+63 at once in a per-wave
// LDS hash table of (position, 4-byte value) entries — the stored value replaces a reload of the
// candidate bytes — and insert them with a 64-bit LDS max so the latest position wins; repeats
// within the window come from comparing each lane with the 32 lanes before it.  A ballot
// picks the first hit (greedy), the match is extended 64 bytes per step by comparing lanes, and the
// sequence is emitted wave-cooperatively.  Windows without a hit cost one gather + one ballot, so
// incompressible bytes (mantissa planes of bf16 weights) stream through.  LZ4 end-of-block rules:
// no match starts in the last 12 bytes, the last 5 bytes are literals.
//
// Two kernels, bit-identical frames:
//   k_lz4_compress_v1  8-byte table entries (position, value), every sequence's bytes stored to HBM
//                      as it is emitted.  32 KiB LDS per wave -> 4 waves per CU, and on gfx9 the
//                      vector memory counter counts stores as well as loads, so each window's
//                      loads after an emit wait for the emit's byte stores to be acknowledged.
//                      rocprof (70B bench setup): 89.7 % of all GPU time, ~3.5 GB/s.
//   k_lz4_compress     (default) 4-byte entries (position << 14 | 14-bit tag of the value; a tag hit
//                      is confirmed by loading the candidate's 4 bytes, so the hit set -- and the
//                      frame -- is exactly v1's) and output staged in a 4 KiB per-wave LDS ring,
//                      written to HBM 2 KiB at a time with coalesced byte stores: the parse's loads
//                      no longer queue behind per-sequence stores, and 20 KiB per wave fits 8 waves
//                      per CU.  ZG_COMPRESS=v1 selects the old kernel (A/B, identity test).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "zgpu.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kTabLog = 12;  // 4096 entries x 8 B = 32 KiB per wave (setup-time kernel: ratio over occupancy)
constexpr uint32_t kTab = 1u << kTabLog;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kWave - 1); }

// 4 bytes at an arbitrary address (aligned dword loads + funnel shift; buffers are padded).
__device__ __forceinline__ uint32_t load_u32(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t k = uint32_t(a & 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t w0 = w[0];
  return k == 0 ? w0 : __builtin_amdgcn_alignbyte(w[1], w0, k);
}

// Lane-parallel write of an LZ4 length continuation (n >= 15 already in the token): 255 x k, rest.
__device__ __forceinline__ uint32_t put_len(uint8_t* o, uint32_t op, uint32_t r, uint32_t lane) {
  const uint32_t nff = r / 255;
  for (uint32_t i = lane; i < nff; i += kWave) o[op + i] = 0xFF;
  if (lane == 0) o[op + nff] = uint8_t(r - 255 * nff);
  return op + nff + 1;
}

// Emit one sequence: literals in[lit0, lit0 + L), then (if ml) a match of ml bytes at distance off.
__device__ __forceinline__ uint32_t emit(uint8_t* o, uint32_t op, const uint8_t* in, uint32_t lit0, uint32_t L,
                                         uint32_t off, uint32_t ml, uint32_t lane) {
  const uint32_t M = ml ? ml - 4 : 0;
  if (lane == 0) o[op] = uint8_t(((L < 15 ? L : 15) << 4) | (ml ? (M < 15 ? M : 15) : 0));
  ++op;
  if (L >= 15) op = put_len(o, op, L - 15, lane);
  for (uint32_t i = lane; i < L; i += kWave) o[op + i] = in[lit0 + i];
  op += L;
  if (ml) {
    if (lane == 0) {
      o[op] = uint8_t(off & 0xFF);
      o[op + 1] = uint8_t(off >> 8);
    }
    op += 2;
    if (M >= 15) op = put_len(o, op, M - 15, lane);
  }
  return op;
}

// BG4 byte grouping of each chunk into its scratch slot: byte i goes to group i % 4.
__global__ void __launch_bounds__(256) k_bg4_split(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ lens, int n, uint8_t* __restrict__ out,
                                                   uint64_t slot) {
  const int c = __builtin_amdgcn_readfirstlane(int(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)));
  if (c >= n) return;
  const uint32_t lane = lane_id(), len = lens[c];
  const uint8_t* s = data + offs[c];
  uint8_t* d = out + uint64_t(c) * slot;
  const uint32_t q = len >> 2, r = len & 3;
  const uint32_t g1 = q + (r > 0), g2 = g1 + q + (r > 1), g3 = g2 + q + (r > 2);
  for (uint32_t i = lane; i < len; i += kWave) {
    const uint32_t g = i & 3, j = i >> 2;
    const uint32_t base = g == 0 ? 0u : g == 1 ? g1 : g == 2 ? g2 : g3;
    d[base + j] = s[i];
  }
}

__global__ void __launch_bounds__(256) k_lz4_compress_v1(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ lens, int n, uint64_t in_slot,
                                                      uint8_t* __restrict__ out, uint64_t out_slot,
                                                      uint32_t* __restrict__ out_len, uint32_t hc64, uint32_t hc256) {
  __shared__ unsigned long long tabs[kWavesPerBlock][kTab];
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int c = __builtin_amdgcn_readfirstlane(int(blockIdx.x * kWavesPerBlock + wave));
  if (c >= n) return;
  const uint32_t lane = lane_id();
  unsigned long long* tab = tabs[wave];
  for (uint32_t i = lane; i < kTab; i += kWave) tab[i] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t len = lens[c];
  // in_slot != 0: input is the BG4 scratch (slot per chunk); else the raw chunk in `data`
  const uint8_t* in = in_slot ? data + uint64_t(c) * in_slot : data + offs[c];
  uint8_t* o = out + uint64_t(c) * out_slot;
  uint32_t op = 11, ip = 0, anchor = 0;
  const uint32_t mend = len > 5 ? len - 5 : 0;  // a match ends at or before len - 5
  while (ip + 12 <= len) {
    const uint32_t p = ip + lane;
    const bool ok = p + 12 <= len;
    const uint32_t v = ok ? load_u32(in + p) : 0;
    const uint32_t h = (v * 2654435761u) >> (32 - kTabLog);
    const unsigned long long e = ok ? tab[h] : 0ull;
    uint32_t cand = uint32_t(e >> 32) - 1;
    bool hit = ok && e != 0 && uint32_t(e) == v && cand < p && p - cand <= 65535u;
    // Repeats closer than the window (runs, short periods) are not in the table yet: compare with
    // the 32 preceding lanes and prefer the nearest equal 4-byte value.
    uint32_t near = 0;
    for (int d = 32; d >= 1; --d) {
      const uint32_t u = __shfl_up(v, d, kWave);
      if (lane >= uint32_t(d) && u == v) near = d;
    }
    if (ok && near) {
      cand = p - near;
      hit = true;
    }
    const unsigned long long mask = __ballot(hit);
    // Insert only the positions the parse moves past (up to the first hit): a later window must
    // never find a position at or beyond its own lanes, which would hide the real candidates.
    const uint32_t passed = mask ? uint32_t(__builtin_ctzll(mask)) + 1 : uint32_t(kWave);
    __builtin_amdgcn_wave_barrier();
    if (ok && lane < passed) atomicMax(&tab[h], (static_cast<unsigned long long>(p + 1) << 32) | v);
    if (!mask) {
      ip += kWave;
      continue;
    }
    const int j = __builtin_ctzll(mask);
    uint32_t mp = ip + uint32_t(j);
    uint32_t mc = uint32_t(__builtin_amdgcn_readlane(int(cand), j));
    // extend backwards over pending literals (64 bytes per step)
    while (true) {
      const uint32_t room = (mp - anchor) < mc ? (mp - anchor) : mc;
      if (room == 0) break;
      const uint32_t k = lane + 1;
      const bool eq = k <= room && in[mp - k] == in[mc - k];
      const unsigned long long ne = __ballot(!eq);
      const uint32_t b = ne ? uint32_t(__builtin_ctzll(ne)) : uint32_t(kWave);
      mp -= b;
      mc -= b;
      if (b < uint32_t(kWave)) break;
    }
    const uint32_t maxlen = mend - mp;  // >= 7 since mp + 12 <= len
    uint32_t ml = 4 + (ip + uint32_t(j) - mp);  // bytes gained backwards are already known to match
    while (ml < maxlen) {
      const uint32_t k = ml + lane;
      const bool eq = k < maxlen && in[mc + k] == in[mp + k];
      const unsigned long long ne = __ballot(!eq);
      if (ne) {
        ml += uint32_t(__builtin_ctzll(ne));
        break;
      }
      ml += kWave;
    }
    if (ml > maxlen) ml = maxlen;
    op = emit(o, op, in, anchor, mp - anchor, mp - mc, ml, lane);
    ip = mp + ml;
    anchor = ip;
  }
  op = emit(o, op, in, anchor, len - anchor, 0, 0, lane);
  const uint32_t total = op + 4;  // + end mark
  if (total >= len) {             // incompressible: the caller stores the chunk raw (scheme 0)
    if (lane == 0) out_len[c] = 0;
    return;
  }
  if (lane == 0) {
    const uint32_t bs = op - 11;
    const bool small = len <= 65536;
    const uint8_t hdr[11] = {0x04, 0x22, 0x4D, 0x18, 0x60, uint8_t(small ? 0x40 : 0x50),
                             uint8_t(small ? hc64 : hc256), uint8_t(bs), uint8_t(bs >> 8), uint8_t(bs >> 16),
                             uint8_t(bs >> 24)};
    for (int i = 0; i < 11; ++i) o[i] = hdr[i];
    for (int i = 0; i < 4; ++i) o[op + i] = 0;
    out_len[c] = total;
  }
}

// ---- k_lz4_compress: compact table + LDS-staged output ----------------------------------------
constexpr uint32_t kTagBits = 14;
constexpr uint32_t kTagMask = (1u << kTagBits) - 1;
constexpr uint32_t kRing = 4096;   // per-wave output staging (bytes)
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kFlush = 2048;  // written to HBM once this many bytes are pending
constexpr uint32_t kHdr = 11;      // frame header bytes, written last (block size known at the end)

// Per-wave staged output: bytes [0, flushed) of the frame are in HBM, [flushed, op) in the ring.
struct Staged {
  uint8_t* ring;
  uint8_t* g;
  uint32_t flushed;
};

// Write ring bytes [flushed, end) to HBM (lane-strided: each store instruction covers 64
// consecutive bytes); header positions are skipped.
__device__ __forceinline__ void ring_write(Staged& o, uint32_t end, uint32_t lane) {
  __builtin_amdgcn_wave_barrier();
  for (uint32_t pos = o.flushed + lane; pos < end; pos += kWave)
    if (pos >= kHdr) o.g[pos] = o.ring[pos & kRingMask];
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void maybe_flush(Staged& o, uint32_t op, uint32_t lane) {
  while (op - o.flushed >= kFlush) {
    ring_write(o, o.flushed + kFlush, lane);
    o.flushed += kFlush;
  }
}

__device__ __forceinline__ uint32_t put_len_s(Staged& o, uint32_t op, uint32_t r, uint32_t lane) {
  const uint32_t nff = r / 255;  // <= 514 for a 128 KiB chunk
  for (uint32_t i = lane; i < nff; i += kWave) o.ring[(op + i) & kRingMask] = 0xFF;
  if (lane == 0) o.ring[(op + nff) & kRingMask] = uint8_t(r - 255 * nff);
  return op + nff + 1;
}

// emit() into the ring.  Pending bytes stay below kRing: a flush check precedes every part that
// can add bytes (token + length <= 516, each literal piece <= 1024, offset + length <= 517).
__device__ __forceinline__ uint32_t emit_s(Staged& o, uint32_t op, const uint8_t* in, uint32_t lit0, uint32_t L,
                                           uint32_t off, uint32_t ml, uint32_t lane) {
  const uint32_t M = ml ? ml - 4 : 0;
  maybe_flush(o, op, lane);
  if (lane == 0) o.ring[op & kRingMask] = uint8_t(((L < 15 ? L : 15) << 4) | (ml ? (M < 15 ? M : 15) : 0));
  ++op;
  if (L >= 15) op = put_len_s(o, op, L - 15, lane);
  for (uint32_t b = 0; b < L; b += 1024) {
    maybe_flush(o, op + b, lane);
    const uint32_t n = L - b < 1024 ? L - b : 1024;
    for (uint32_t i = lane; i < n; i += kWave) o.ring[(op + b + i) & kRingMask] = in[lit0 + b + i];
  }
  op += L;
  if (ml) {
    maybe_flush(o, op, lane);
    if (lane == 0) {
      o.ring[op & kRingMask] = uint8_t(off & 0xFF);
      o.ring[(op + 1) & kRingMask] = uint8_t(off >> 8);
    }
    op += 2;
    if (M >= 15) op = put_len_s(o, op, M - 15, lane);
  }
  return op;
}

__global__ void __launch_bounds__(256) k_lz4_compress(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ lens, int n, uint64_t in_slot,
                                                      uint8_t* __restrict__ out, uint64_t out_slot,
                                                      uint32_t* __restrict__ out_len, uint32_t hc64, uint32_t hc256) {
  __shared__ uint32_t tabs[kWavesPerBlock][kTab];
  __shared__ uint8_t rings[kWavesPerBlock][kRing];
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int c = __builtin_amdgcn_readfirstlane(int(blockIdx.x * kWavesPerBlock + wave));
  if (c >= n) return;
  const uint32_t lane = lane_id();
  uint32_t* tab = tabs[wave];
  for (uint32_t i = lane; i < kTab; i += kWave) tab[i] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t len = lens[c];
  const uint8_t* in = in_slot ? data + uint64_t(c) * in_slot : data + offs[c];
  Staged o{rings[wave], out + uint64_t(c) * out_slot, 0};
  uint32_t op = kHdr, ip = 0, anchor = 0;
  const uint32_t mend = len > 5 ? len - 5 : 0;
  while (ip + 12 <= len) {
    const uint32_t p = ip + lane;
    const bool ok = p + 12 <= len;
    const uint32_t v = ok ? load_u32(in + p) : 0;
    const uint32_t hv = v * 2654435761u;
    const uint32_t h = hv >> (32 - kTabLog);
    const uint32_t tag = hv & kTagMask;
    const uint32_t e = ok ? tab[h] : 0u;
    uint32_t cand = (e >> kTagBits) - 1;
    bool hit = ok && e != 0 && (e & kTagMask) == tag && cand < p && p - cand <= 65535u;
    if (hit) hit = load_u32(in + cand) == v;  // the tag matched: confirm the value (v1 stored it)
    uint32_t near = 0;
    for (int d = 32; d >= 1; --d) {
      const uint32_t u = __shfl_up(v, d, kWave);
      if (lane >= uint32_t(d) && u == v) near = d;
    }
    if (ok && near) {
      cand = p - near;
      hit = true;
    }
    const unsigned long long mask = __ballot(hit);
    const uint32_t passed = mask ? uint32_t(__builtin_ctzll(mask)) + 1 : uint32_t(kWave);
    __builtin_amdgcn_wave_barrier();
    if (ok && lane < passed) atomicMax(&tab[h], ((p + 1) << kTagBits) | tag);
    if (!mask) {
      ip += kWave;
      continue;
    }
    const int j = __builtin_ctzll(mask);
    uint32_t mp = ip + uint32_t(j);
    uint32_t mc = uint32_t(__builtin_amdgcn_readlane(int(cand), j));
    while (true) {
      const uint32_t room = (mp - anchor) < mc ? (mp - anchor) : mc;
      if (room == 0) break;
      const uint32_t k = lane + 1;
      const bool eq = k <= room && in[mp - k] == in[mc - k];
      const unsigned long long ne = __ballot(!eq);
      const uint32_t b = ne ? uint32_t(__builtin_ctzll(ne)) : uint32_t(kWave);
      mp -= b;
      mc -= b;
      if (b < uint32_t(kWave)) break;
    }
    const uint32_t maxlen = mend - mp;
    uint32_t ml = 4 + (ip + uint32_t(j) - mp);
    while (ml < maxlen) {
      const uint32_t k = ml + lane;
      const bool eq = k < maxlen && in[mc + k] == in[mp + k];
      const unsigned long long ne = __ballot(!eq);
      if (ne) {
        ml += uint32_t(__builtin_ctzll(ne));
        break;
      }
      ml += kWave;
    }
    if (ml > maxlen) ml = maxlen;
    op = emit_s(o, op, in, anchor, mp - anchor, mp - mc, ml, lane);
    ip = mp + ml;
    anchor = ip;
  }
  op = emit_s(o, op, in, anchor, len - anchor, 0, 0, lane);
  const uint32_t total = op + 4;
  if (total >= len) {
    if (lane == 0) out_len[c] = 0;
    return;
  }
  maybe_flush(o, op, lane);
  if (lane < 4) o.ring[(op + lane) & kRingMask] = 0;  // end mark
  ring_write(o, total, lane);
  if (lane == 0) {
    const uint32_t bs = op - kHdr;
    const bool small = len <= 65536;
    const uint8_t hdr[kHdr] = {0x04, 0x22, 0x4D, 0x18, 0x60, uint8_t(small ? 0x40 : 0x50),
                               uint8_t(small ? hc64 : hc256), uint8_t(bs), uint8_t(bs >> 8), uint8_t(bs >> 16),
                               uint8_t(bs >> 24)};
    for (uint32_t i = 0; i < kHdr; ++i) o.g[i] = hdr[i];
    out_len[c] = total;
  }
}

bool compress_v1() {  // read per launch (a setup-time kernel), so a test can A/B both in one process
  const char* e = getenv("ZG_COMPRESS");
  return e && e[0] == 'v' && e[1] == '1';
}

// Serialize chunks as xorb body entries: 8-byte header [0][clen u24][scheme][ulen u24] + payload
// copied from an arbitrary device address per chunk (compressed frame or raw chunk).
__global__ void __launch_bounds__(256) k_pack_frames(const uint64_t* __restrict__ src, const uint32_t* __restrict__ clen,
                                                     const uint32_t* __restrict__ ulen, const uint8_t* __restrict__ scheme,
                                                     const uint64_t* __restrict__ out_off, int n, uint8_t* __restrict__ out) {
  const int c = __builtin_amdgcn_readfirstlane(int(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)));
  if (c >= n) return;
  const uint32_t lane = lane_id(), cl = clen[c], ul = ulen[c];
  uint8_t* d = out + out_off[c];
  if (lane < 8) {
    const uint32_t b = lane == 0 ? 0u : lane < 4 ? (cl >> (8 * (lane - 1))) & 0xFF
                                  : lane == 4 ? scheme[c] : (ul >> (8 * (lane - 5))) & 0xFF;
    d[lane] = uint8_t(b);
  }
  const uint8_t* s = reinterpret_cast<const uint8_t*>(src[c]);
  for (uint32_t i = lane; i < cl; i += kWave) d[8 + i] = s[i];
}

}  // namespace

extern "C" {

hipError_t zg_compress_chunks(const uint8_t* data, const uint64_t* offs, const uint32_t* lens, int n, int bg4,
                              uint8_t* scratch, uint64_t in_slot, uint8_t* out, uint64_t out_slot, uint32_t* out_len,
                              uint32_t hc64, uint32_t hc256, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + kWavesPerBlock - 1) / kWavesPerBlock);
  auto* kern = compress_v1() ? k_lz4_compress_v1 : k_lz4_compress;
  if (bg4) {
    hipLaunchKernelGGL(k_bg4_split, grid, dim3(256), 0, stream, data, offs, lens, n, scratch, in_slot);
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, scratch, offs, lens, n, in_slot, out, out_slot, out_len,
                       hc64, hc256);
  } else {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, data, offs, lens, n, uint64_t(0), out, out_slot, out_len,
                       hc64, hc256);
  }
  return hipGetLastError();
}

hipError_t zg_pack_frames(const uint64_t* src, const uint32_t* clen, const uint32_t* ulen, const uint8_t* scheme,
                          const uint64_t* out_off, int n, uint8_t* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack_frames, dim3((n + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, stream, src, clen,
                     ulen, scheme, out_off, n, out);
  return hipGetLastError();
}

}  // extern "C"
