// Xorb ingest kernels for MI355X (gfx950, CDNA4, wave64): index -> place (copy / LZ4 decode)
// -> hash.  SURVEY §2.G K1 (BLAKE3 chunk hashes), K3 (LZ4/BG4 decode), K4 (header walk + fused
// ingest).  Host oracle: csrc/core/{xorb,lz4,blake3}.cpp.
//
// Buffers handed to these kernels must be padded by >= 4 KiB past their logical end: the
// alignment-fixing loads read whole aligned dwords (and the LZ4 window reads 256-byte lines).
#include <hip/hip_runtime.h>

#include "blake3_dev.h"
#include "zgpu.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr uint32_t kMaxChunk = 128u * 1024u;  // Xet CDC maximum chunk size

__device__ __forceinline__ void report(unsigned long long* err, uint32_t code, uint32_t idx) {
  if (err) atomicCAS(err, 0ull, (static_cast<unsigned long long>(code) << 32) | idx);
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Load 8 bytes at an arbitrary address as two little-endian words (reads aligned dwords).
__device__ __forceinline__ void load8(const uint8_t* p, uint32_t& lo, uint32_t& hi) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t k = uint32_t(a & 3);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t w0 = w[0], w1 = w[1];
  if (k == 0) {
    lo = w0;
    hi = w1;
  } else {
    const uint32_t w2 = w[2];
    lo = __builtin_amdgcn_alignbyte(w1, w0, k);
    hi = __builtin_amdgcn_alignbyte(w2, w1, k);
  }
}

// --------------------------------------------------------------------------------------------
// K4a: header walk.  One thread per fetched run; sequential by construction (chunk i+1's header
// position depends on chunk i's compressed length), parallel across runs.
// --------------------------------------------------------------------------------------------
__global__ void k_index_terms(const uint8_t* __restrict__ src, const ZgTerm* __restrict__ terms, int n_terms,
                              ZgChunk* __restrict__ chunks, unsigned long long* err) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_terms) return;
  const ZgTerm tm = terms[t];
  const uint8_t* p = src + tm.src;
  uint64_t off = 0, uoff = 0;
  // On any error the remaining descriptors of this term are written as empty no-ops so later
  // kernels never dereference garbage.
  auto fail = [&](uint32_t code, uint32_t from) {
    report(err, code, uint32_t(t));
    ZgChunk z{0, 0, 0, 0, 0, uint32_t(t)};
    for (uint32_t k = from; k < tm.n_chunks; ++k) chunks[tm.chunk_base + k] = z;
  };
  for (uint32_t c = 0; c < tm.n_chunks; ++c) {
    if (off + 8 > tm.src_len) {
      fail(ZG_ERR_COUNT, c);
      return;
    }
    uint32_t lo, hi;
    load8(p + off, lo, hi);
    const uint32_t version = lo & 0xFF;
    const uint32_t clen = lo >> 8;
    const uint32_t scheme = hi & 0xFF;
    const uint32_t ulen = hi >> 8;
    if (version != 0 || scheme > 2 || (scheme == 0 && clen != ulen)) {
      fail(ZG_ERR_HEADER, c);
      return;
    }
    if (off + 8 + clen > tm.src_len || (tm.ulen != 0 && uoff + ulen > tm.ulen)) {
      fail(ZG_ERR_RANGE, c);
      return;
    }
    if (ulen > kMaxChunk) {
      fail(ZG_ERR_CAPACITY, c);
      return;
    }
    ZgChunk ch;
    ch.src = tm.src + off + 8;
    ch.dst = tm.dst + uoff;
    ch.clen = clen;
    ch.ulen = ulen;
    ch.scheme = scheme;
    ch.term = uint32_t(t);
    chunks[tm.chunk_base + c] = ch;
    off += 8 + clen;
    uoff += ulen;
  }
  if (off != tm.src_len || (tm.ulen != 0 && uoff != tm.ulen)) report(err, ZG_ERR_COUNT, uint32_t(t));
}

// --------------------------------------------------------------------------------------------
// Wave-cooperative byte-exact copy between arbitrarily aligned addresses: 16-byte aligned
// dwordx4 stores; the source is read as aligned dwords and funnel-shifted (v_alignbyte_b32).
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_copy(uint8_t* d, const uint8_t* s, uint64_t n, uint32_t lane) {
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

// K3a: place uncompressed chunks (scheme 0): one wave per chunk, clipped to [clip_lo, clip_hi).
__global__ void __launch_bounds__(256) k_place_raw(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   const ZgChunk* __restrict__ chunks, int n_chunks,
                                                   uint64_t clip_lo, uint64_t clip_hi, uint64_t src_n,
                                                   uint64_t dst_n) {
  const int c = wave_uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  if (c >= n_chunks) return;
  const ZgChunk ch = chunks[c];
  if (ch.scheme != 0) return;
  if (ch.src + ch.ulen > src_n || ch.dst + ch.ulen > dst_n) return;
  const uint64_t lo = ch.dst > clip_lo ? ch.dst : clip_lo;
  const uint64_t end = ch.dst + ch.ulen;
  const uint64_t hi = end < clip_hi ? end : clip_hi;
  if (lo >= hi) return;
  wave_copy(dst + lo, src + ch.src + (lo - ch.dst), hi - lo, lane_id());
}

// --------------------------------------------------------------------------------------------
// K3b: LZ4-frame (+BG4) decode.  One wave per chunk, output assembled in LDS, then written to
// HBM with the BG4 regroup fused into the store pass.  Token parsing reads a 256-byte window of
// the compressed stream held one dword per lane (v_readlane_b32), literal bytes are fetched from
// that window with ds_bpermute, match copies run lane-parallel in LDS (overlapping matches use
// the periodic form out[op+i] = out[op-off+(i mod off)], so every source byte is final).
// --------------------------------------------------------------------------------------------
struct Window {
  uintptr_t base;  // absolute, 4-byte aligned
  uint32_t w;      // this lane's dword: bytes [base + 4*lane, +4)
};

__device__ __forceinline__ void win_fill(Window& win, uintptr_t addr, uint32_t lane) {
  win.base = addr & ~uintptr_t(3);
  win.w = reinterpret_cast<const uint32_t*>(win.base)[lane];
}

// Ensure [a, a + need) is inside the window (need <= 252).
__device__ __forceinline__ void win_ensure(Window& win, uintptr_t a, uint32_t need, uint32_t lane) {
  if (a < win.base || a + need > win.base + 256) win_fill(win, a, lane);
}

// Uniform byte read (a must be inside the window).
__device__ __forceinline__ uint32_t win_byte(const Window& win, uintptr_t a) {
  const uint32_t rel = uint32_t(a - win.base);
  const uint32_t w = __builtin_amdgcn_readlane(win.w, int(rel >> 2));
  return (w >> (8 * (rel & 3))) & 0xFF;
}

// Per-lane byte read: lane i gets the byte at a + i (a + 64 must be inside the window).
__device__ __forceinline__ uint32_t win_lane_byte(const Window& win, uintptr_t a, uint32_t lane) {
  const uint32_t rel = uint32_t(a - win.base) + lane;
  const uint32_t w = __shfl(win.w, int(rel >> 2), kWave);
  return (w >> (8 * (rel & 3))) & 0xFF;
}

// Decode one LZ4 block (blk[0..blen)) into lds at op; returns new op, or ~0u on error.
__device__ uint32_t lz4_block(Window& win, uintptr_t blk, uint32_t blen, uint8_t* lds, uint32_t op,
                              uint32_t cap, uint32_t lane) {
  uint32_t bp = 0;
  while (true) {
    if (bp >= blen) return ~0u;
    win_ensure(win, blk + bp, 32, lane);
    const uint32_t token = win_byte(win, blk + bp);
    ++bp;
    uint32_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (bp >= blen) return ~0u;
        win_ensure(win, blk + bp, 1, lane);
        b = win_byte(win, blk + bp);
        ++bp;
        lit += b;
      } while (b == 255);
    }
    if (lit > blen - bp || lit > cap - op) return ~0u;
    for (uint32_t i = 0; i < lit; i += kWave) {
      win_ensure(win, blk + bp + i, kWave, lane);
      const uint32_t v = win_lane_byte(win, blk + bp + i, lane);
      if (i + lane < lit) lds[op + i + lane] = uint8_t(v);
    }
    bp += lit;
    op += lit;
    if (bp == blen) return op;
    if (blen - bp < 2) return ~0u;
    win_ensure(win, blk + bp, 32, lane);
    const uint32_t off = win_byte(win, blk + bp) | (win_byte(win, blk + bp + 1) << 8);
    bp += 2;
    if (off == 0 || off > op) return ~0u;
    uint32_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (bp >= blen) return ~0u;
        win_ensure(win, blk + bp, 1, lane);
        b = win_byte(win, blk + bp);
        ++bp;
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (ml > cap - op) return ~0u;
    if (off >= ml) {
      for (uint32_t i = lane; i < ml; i += kWave) lds[op + i] = lds[op - off + i];
    } else {
      for (uint32_t i = lane; i < ml; i += kWave) lds[op + i] = lds[op - off + (i % off)];
    }
    op += ml;
  }
}

// Returns decoded length or ~0u on malformed frame.
__device__ uint32_t lz4_frame(const uint8_t* payload, uint32_t clen, uint8_t* lds, uint32_t cap, uint32_t lane) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(payload);
  Window win;
  win_fill(win, p, lane);
  if (clen < 7) return ~0u;
  const uint32_t magic = win_byte(win, p) | (win_byte(win, p + 1) << 8) | (win_byte(win, p + 2) << 16) |
                         (win_byte(win, p + 3) << 24);
  if (magic != 0x184D2204u) return ~0u;
  const uint32_t flg = win_byte(win, p + 4);
  if ((flg >> 6) != 1) return ~0u;
  uint32_t ip = 7 + ((flg & 8) ? 8 : 0) + ((flg & 1) ? 4 : 0);
  const bool block_ck = flg & 0x10;
  uint32_t op = 0;
  while (true) {
    if (clen - ip < 4 || ip > clen) return ~0u;
    win_ensure(win, p + ip, 4, lane);
    const uint32_t bs = win_byte(win, p + ip) | (win_byte(win, p + ip + 1) << 8) |
                        (win_byte(win, p + ip + 2) << 16) | (win_byte(win, p + ip + 3) << 24);
    ip += 4;
    if (bs == 0) break;
    const uint32_t len = bs & 0x7FFFFFFFu;
    if (len > clen - ip) return ~0u;
    if (bs & 0x80000000u) {
      if (len > cap - op) return ~0u;
      for (uint32_t i = 0; i < len; i += kWave) {
        win_ensure(win, p + ip + i, kWave, lane);
        const uint32_t v = win_lane_byte(win, p + ip + i, lane);
        if (i + lane < len) lds[op + i + lane] = uint8_t(v);
      }
      op += len;
    } else {
      op = lz4_block(win, p + ip, len, lds, op, cap, lane);
      if (op == ~0u) return ~0u;
    }
    ip += len + (block_ck ? 4 : 0);
  }
  return op;
}

// Store LDS chunk bytes to dst[lo, hi) (chunk-relative [lo - base, hi - base)), applying the
// BG4 regroup when `bg4`: original byte j = grouped[goff[j & 3] + (j >> 2)].
__device__ void store_from_lds(const uint8_t* lds, uint32_t ulen, bool bg4, uint8_t* dst_chunk, uint32_t lo,
                               uint32_t hi, uint32_t lane) {
  const uint32_t q = ulen >> 2, r = ulen & 3;
  const uint32_t g1 = q + (r > 0 ? 1 : 0);
  const uint32_t g2 = g1 + q + (r > 1 ? 1 : 0);
  const uint32_t g3 = g2 + q + (r > 2 ? 1 : 0);
  auto src_of = [&](uint32_t j) -> uint32_t {
    if (!bg4) return j;
    const uint32_t g = j & 3, i = j >> 2;
    const uint32_t base = g == 0 ? 0 : g == 1 ? g1 : g == 2 ? g2 : g3;
    return base + i;
  };
  // head bytes until dst 4-aligned
  const uintptr_t da = reinterpret_cast<uintptr_t>(dst_chunk + lo);
  uint32_t head = uint32_t((4 - (da & 3)) & 3);
  if (head > hi - lo) head = hi - lo;
  if (lane < head) dst_chunk[lo + lane] = lds[src_of(lo + lane)];
  const uint32_t s = lo + head;
  const uint32_t nw = (hi - s) >> 2;
  uint32_t* dw = reinterpret_cast<uint32_t*>(dst_chunk + s);
  for (uint32_t w = lane; w < nw; w += kWave) {
    const uint32_t j = s + 4 * w;
    uint32_t v;
    if (!bg4) {
      v = uint32_t(lds[j]) | (uint32_t(lds[j + 1]) << 8) | (uint32_t(lds[j + 2]) << 16) | (uint32_t(lds[j + 3]) << 24);
    } else {
      v = uint32_t(lds[src_of(j)]) | (uint32_t(lds[src_of(j + 1)]) << 8) | (uint32_t(lds[src_of(j + 2)]) << 16) |
          (uint32_t(lds[src_of(j + 3)]) << 24);
    }
    dw[w] = v;
  }
  const uint32_t t = s + 4 * nw;
  if (lane < hi - t) dst_chunk[t + lane] = lds[src_of(t + lane)];
}

__global__ void __launch_bounds__(64) k_decode_lz4(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   const ZgChunk* __restrict__ chunks, int n_chunks,
                                                   uint64_t clip_lo, uint64_t clip_hi, unsigned long long* err,
                                                   uint32_t lds_cap, uint64_t src_n, uint64_t dst_n) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t lane = lane_id();
  for (int c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const ZgChunk ch = chunks[c];
    if (ch.scheme == 0) continue;
    if (ch.src + ch.clen > src_n || ch.dst + ch.ulen > dst_n) {
      report(err, ZG_ERR_RANGE, uint32_t(c));
      continue;
    }
    const uint64_t lo = ch.dst > clip_lo ? ch.dst : clip_lo;
    const uint64_t end = ch.dst + ch.ulen;
    const uint64_t hi = end < clip_hi ? end : clip_hi;
    if (lo >= hi) continue;
    if (ch.ulen > lds_cap) {
      report(err, ZG_ERR_CAPACITY, uint32_t(c));
      continue;
    }
    const uint32_t got = lz4_frame(src + ch.src, ch.clen, lds, ch.ulen, lane);
    if (got == ~0u) {
      report(err, ZG_ERR_LZ4, uint32_t(c));
      continue;
    }
    if (got != ch.ulen) {
      report(err, ZG_ERR_SIZE, uint32_t(c));
      continue;
    }
    store_from_lds(lds, ch.ulen, ch.scheme == 2, dst + ch.dst, uint32_t(lo - ch.dst), uint32_t(hi - ch.dst), lane);
  }
}

// --------------------------------------------------------------------------------------------
// K1: keyed BLAKE3 chunk hashes.  One wave per Xet chunk (4 per 256-thread block); lane l owns
// BLAKE3 chunks l, l+64 (<= 128 for a 128 KiB Xet chunk); chaining values are merged pairwise
// in LDS (pairwise-with-carry == BLAKE3's left-complete tree).
// --------------------------------------------------------------------------------------------
__device__ void wave_hash(const uint8_t* base, uint32_t len, const zg::Key8& key, uint32_t mode, uint32_t* cvs,
                          uint32_t lane, uint32_t out[8]) {
  const uint32_t nb = len == 0 ? 1 : (len + 1023) >> 10;
  if (nb == 1) {
    uint32_t cv[8];
    if (lane == 0) zg::hash_chunk(base, len, 0, key, mode, true, cv);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = __builtin_amdgcn_readfirstlane(cv[i]);
    return;
  }
  for (uint32_t b = lane; b < nb; b += kWave) {
    const uint32_t seg = len - (b << 10) < 1024 ? len - (b << 10) : 1024;
    uint32_t cv[8];
    zg::hash_chunk(base + (size_t(b) << 10), seg, b, key, mode, false, cv);
#pragma unroll
    for (int i = 0; i < 8; ++i) cvs[8 * b + i] = cv[i];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t m = nb;
  while (m > 2) {
    const uint32_t pairs = m >> 1;
    for (uint32_t i = lane; i < pairs; i += kWave) {
      uint32_t l[8], r[8], o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        l[k] = cvs[16 * i + k];
        r[k] = cvs[16 * i + 8 + k];
      }
      zg::parent_cv(l, r, key, mode, false, o);
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
  zg::parent_cv(l, r, key, mode, true, o);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = o[k];
}

__device__ __forceinline__ void store_hash(uint8_t* dst, const uint32_t h[8], uint32_t lane) {
  if (lane < 8) reinterpret_cast<uint32_t*>(dst)[lane] = h[0] * (lane == 0) + h[1] * (lane == 1) + h[2] * (lane == 2) +
                                                          h[3] * (lane == 3) + h[4] * (lane == 4) + h[5] * (lane == 5) +
                                                          h[6] * (lane == 6) + h[7] * (lane == 7);
}

__global__ void __launch_bounds__(256) k_hash_chunks(const uint8_t* __restrict__ dst, const ZgChunk* __restrict__ chunks,
                                                     int n_chunks, uint8_t* __restrict__ hashes,
                                                     uint64_t* __restrict__ sizes, uint32_t hash_index_base,
                                                     uint64_t dst_n) {
  __shared__ uint32_t cvs_all[kWavesPerBlock][128 * 8];
  const int wid = threadIdx.x >> 6;
  const int c = wave_uniform(blockIdx.x * kWavesPerBlock + wid);
  if (c >= n_chunks) return;
  const uint32_t lane = lane_id();
  ZgChunk ch = chunks[c];
  if (ch.dst + ch.ulen > dst_n || ch.ulen > kMaxChunk) ch.ulen = 0, ch.dst = 0;
  uint32_t h[8];
  wave_hash(dst + ch.dst, ch.ulen, zg::kDataKeyW, zg::KEYED_HASH, cvs_all[wid], lane, h);
  const uint64_t idx = uint64_t(hash_index_base) + uint64_t(c);
  store_hash(hashes + 32 * idx, h, lane);
  if (sizes && lane == 0) sizes[idx] = ch.ulen;
}

__global__ void __launch_bounds__(256) k_hash_ranges(const uint8_t* __restrict__ buf, const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens, int n, uint8_t* __restrict__ out,
                                                     int key_mode) {
  __shared__ uint32_t cvs_all[kWavesPerBlock][128 * 8];
  const int wid = threadIdx.x >> 6;
  const int c = wave_uniform(blockIdx.x * kWavesPerBlock + wid);
  if (c >= n) return;
  const uint32_t lane = lane_id();
  const uint32_t len = lens[c];
  uint32_t h[8];
  if (len > 128u * 1024u) {
    if (lane < 8) reinterpret_cast<uint32_t*>(out + 32 * size_t(c))[lane] = 0xFFFFFFFFu;
    return;
  }
  const zg::Key8& key = key_mode == 0 ? zg::kDataKeyW : key_mode == 1 ? zg::kNodeKeyW : key_mode == 2 ? zg::kIVW : zg::kZeroW;
  const uint32_t mode = key_mode == 2 ? 0u : zg::KEYED_HASH;
  wave_hash(buf + offs[c], len, key, mode, cvs_all[wid], lane, h);
  store_hash(out + 32 * size_t(c), h, lane);
}

__global__ void k_compare(const uint8_t* __restrict__ got, const uint8_t* __restrict__ want, int n,
                          unsigned long long* err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* a = reinterpret_cast<const uint4*>(got + 32 * size_t(i));
  const uint4* b = reinterpret_cast<const uint4*>(want + 32 * size_t(i));
  const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
  if (a0.x != b0.x || a0.y != b0.y || a0.z != b0.z || a0.w != b0.w || a1.x != b1.x || a1.y != b1.y ||
      a1.z != b1.z || a1.w != b1.w)
    report(err, ZG_ERR_HASH, uint32_t(i));
}

}  // namespace

extern "C" {

hipError_t zg_index_terms(const uint8_t* src, const ZgTerm* terms, int n_terms, ZgChunk* chunks,
                          unsigned long long* err, hipStream_t stream) {
  if (n_terms <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_index_terms, dim3((n_terms + 63) / 64), dim3(64), 0, stream, src, terms, n_terms, chunks, err);
  return hipGetLastError();
}

hipError_t zg_place_chunks(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                           int n_chunks, uint64_t clip_lo, uint64_t clip_hi, unsigned long long* err,
                           hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_place_raw, dim3((n_chunks + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, stream, src,
                     dst, chunks, n_chunks, clip_lo, clip_hi, src_n, dst_n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t cap = kMaxChunk;
  const size_t lds = cap + 16;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(k_decode_lz4), hipFuncAttributeMaxDynamicSharedMemorySize,
                        int(lds));
    attr_set = true;
  }
  const int grid = n_chunks < 1024 ? n_chunks : 1024;
  hipLaunchKernelGGL(k_decode_lz4, dim3(grid), dim3(64), lds, stream, src, dst, chunks, n_chunks, clip_lo, clip_hi,
                     err, cap, src_n, dst_n);
  return hipGetLastError();
}

hipError_t zg_hash_chunks(const uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks, int n_chunks, uint8_t* hashes,
                          uint64_t* sizes, uint32_t hash_index_base, hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hash_chunks, dim3((n_chunks + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, stream, dst,
                     chunks, n_chunks, hashes, sizes, hash_index_base, dst_n);
  return hipGetLastError();
}

hipError_t zg_hash_ranges(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lens, int n, uint8_t* hashes,
                          int key_mode, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hash_ranges, dim3((n + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, stream, buf, offsets,
                     lens, n, hashes, key_mode);
  return hipGetLastError();
}

hipError_t zg_compare_hashes(const uint8_t* got, const uint8_t* want, int n, unsigned long long* err,
                             hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_compare, dim3((n + 255) / 256), dim3(256), 0, stream, got, want, n, err);
  return hipGetLastError();
}

int zg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
