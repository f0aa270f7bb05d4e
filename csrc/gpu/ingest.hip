// Xorb ingest kernels for MI355X (gfx950, CDNA4, wave64): index -> place (copy / LZ4 decode)
// -> hash.  SURVEY §2.G K1 (BLAKE3 chunk hashes), K3 (LZ4/BG4 decode), K4 (header walk + fused
// ingest).  Host oracle: csrc/core/{xorb,lz4,blake3}.cpp.
//
// Buffers handed to these kernels must be padded by >= 4 KiB past their logical end: the
// alignment-fixing loads read whole aligned dwords (and the LZ4 window reads 256-byte lines).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "blake3_dev.h"
#include "lz4win.h"
#include "wave64.h"
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
// The walk of one run: `hdr(off, lo, hi)` yields the 8 header bytes at run offset `off` (a global
// load, or a lookup in a table the scan below built).  On any error the remaining descriptors of
// the term are written as empty no-ops so later kernels never dereference garbage.
template <class Hdr>
__device__ __forceinline__ void walk_term(const ZgTerm& tm, int t, ZgChunk* __restrict__ chunks, unsigned long long* err,
                                          const Hdr& hdr) {
  uint64_t off = 0, uoff = 0;
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
    hdr(off, lo, hi);
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

struct GlobalHdr {
  const uint8_t* p;
  __device__ __forceinline__ void operator()(uint64_t off, uint32_t& lo, uint32_t& hi) const { load8(p + off, lo, hi); }
};

__global__ void k_index_terms(const uint8_t* __restrict__ src, const ZgTerm* __restrict__ terms, int n_terms,
                              ZgChunk* __restrict__ chunks, unsigned long long* err) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_terms) return;
  const ZgTerm tm = terms[t];
  walk_term(tm, t, chunks, err, GlobalHdr{src + tm.src});
}

// K4a': parallel header walk ("scan, sort, link").  The walk above is one dependent HBM load per
// chunk: ~1000 chained loads per 64 MiB xorb run, ~0.6 ms whatever the GPU's width.  Here:
//   scan   every byte position of the span is tested in parallel for a plausible chunk header
//          (version 0, scheme <= 2, 1 <= ulen <= 128 KiB, clen >= 1, raw => clen == ulen, payload
//          inside its run, a compressed payload starting with the LZ4 frame magic); candidates
//          (one per chunk, plus a few look-alikes per 256 MiB) are appended to their term's list.
//   link   one workgroup per term sorts its candidates in LDS (bitonic), picks the chain from
//          offset 0 to the run's end out of them (successor lookups, see k_hdr_link) and checks
//          it has n_chunks links; block prefix sums give every chunk's index and output offset and
//          the records are written in parallel.
// Anything else -- a list over capacity, a broken, ambiguous or short chain -- falls back to the
// serial walk for that term, so records and error codes are exactly walk_term's.
constexpr int kScanThreads = 256;
// 64 positions per thread from 80 loaded bytes (5 x 16 B): 1.25 loads per position byte instead of
// 2 with 16 positions from 32 bytes
constexpr uint32_t kScanBytesPerThread = 64;
constexpr uint32_t kScanWords = (kScanBytesPerThread + 16) / 4;
constexpr uint32_t kCandCap = 8192;  // chunks of a 64 MiB xorb at the 8 KiB CDC minimum
constexpr int kLinkThreads = 1024;

// `pay`: the 4 bytes after the header.  A compressed chunk's payload is an LZ4 frame, so it starts
// with the frame magic: without that test the LZ4 streams of BG4 bf16 weights (zero bytes every few
// bytes) produced millions of header-like candidates and the scan lost to the serial walk.
constexpr uint32_t kLz4Magic = 0x184D2204u;
__device__ __forceinline__ bool plausible_header(uint32_t lo, uint32_t hi, uint32_t pay, uint64_t rel,
                                                 uint64_t run_len) {
  const uint32_t clen = lo >> 8, scheme = hi & 0xFF, ulen = hi >> 8;
  return (lo & 0xFF) == 0 && scheme <= 2 && ulen >= 1 && ulen <= kMaxChunk && clen >= 1 &&
         (scheme == 0 ? clen == ulen : pay == kLz4Magic) && rel + 8 + clen <= run_len;
}

// terms must be sorted by src (else the fast path finds no chain and the serial walk runs)
__global__ void __launch_bounds__(kScanThreads) k_hdr_scan(const uint8_t* __restrict__ src, uint64_t src_n,
                                                          const ZgTerm* __restrict__ terms, int n_terms,
                                                          uint32_t* __restrict__ counts, uint32_t* __restrict__ cands) {
  const uint64_t q = (uint64_t(blockIdx.x) * kScanThreads + threadIdx.x) * kScanBytesPerThread;
  if (q >= src_n) return;
  // the last term starting at or before q (binary search; terms are few)
  int lo_t = 0, hi_t = n_terms - 1, t = -1;
  while (lo_t <= hi_t) {
    const int mid = (lo_t + hi_t) >> 1;
    if (terms[mid].src <= q) {
      t = mid;
      lo_t = mid + 1;
    } else {
      hi_t = mid - 1;
    }
  }
  if (t < 0) {
    t = 0;  // q lies before the first term: positions below terms[0].src are skipped
  }
  uint64_t t0 = terms[t].src, t1 = t0 + terms[t].src_len;
  uint64_t nx = t + 1 < n_terms ? terms[t + 1].src : ~uint64_t(0);
  uint32_t w[kScanWords];
#pragma unroll
  for (uint32_t i = 0; i < kScanWords / 4; ++i) {  // padded buffers: safe past the end
    const uint4 v = *reinterpret_cast<const uint4*>(src + q + 16 * i);
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
#pragma unroll
  for (uint32_t k = 0; k < kScanBytesPerThread; ++k) {
    const uint64_t p = q + k;
    while (p >= nx) {  // crossed into the next term (wave-divergent, rare)
      ++t;
      t0 = terms[t].src;
      t1 = t0 + terms[t].src_len;
      nx = t + 1 < n_terms ? terms[t + 1].src : ~uint64_t(0);
    }
    if (p < t0 || p + 8 > t1) continue;
    const uint32_t j = k >> 2, sh = k & 3;
    const uint32_t lo = sh ? __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh) : w[j];
    const uint32_t hi = sh ? __builtin_amdgcn_alignbyte(w[j + 2], w[j + 1], sh) : w[j + 1];
    const uint32_t pay = sh ? __builtin_amdgcn_alignbyte(w[j + 3], w[j + 2], sh) : w[j + 2];
    if (plausible_header(lo, hi, pay, p - t0, t1 - t0)) {
      const uint32_t i = atomicAdd(&counts[t], 1u);
      if (i < kCandCap) cands[uint64_t(t) * kCandCap + i] = uint32_t(p - t0);
    }
  }
}

// Link.  The candidates are sorted, then every candidate's successor (its offset + 8 + clen) is
// looked up among them.  False candidates do occur: LZ4 streams of BG4 bf16 weights hold a few
// raw-header look-alikes ([00 x y z 00 x y z], clen == ulen) per 256 MiB, so demanding exactly
// n_chunks candidates sent every term of a 256 MiB batch back to the serial walk.  The chain is
// instead picked out of the candidate set G' = {candidates with a successor (a candidate, or the
// run's end) that sit at offset 0 or are some candidate's successor}.  If G' contains offset 0, is
// closed under the successor, and has exactly n_chunks members, it IS the true chain: the true
// chain starts at 0 and follows successors, so closure puts all of it in G', and the count leaves
// room for nothing else.  Otherwise the serial walk decides (records and error codes stay exactly
// walk_term's).
constexpr uint32_t kEnd = 0xFFFFFFFEu, kNone = 0xFFFFFFFFu;
constexpr uint32_t kPointed = 1u << 31, kGood = 1u << 30;
constexpr uint32_t kFellBack = 1u << 31;  // in counts[t] after the link: term t took the serial walk

__device__ __forceinline__ uint32_t lds_find(const uint32_t* key, uint32_t n, uint32_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (key[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && key[lo] == v ? lo : kNone;
}

__global__ void __launch_bounds__(kLinkThreads) k_hdr_link(const uint8_t* __restrict__ src,
                                                          const ZgTerm* __restrict__ terms,
                                                          uint32_t* __restrict__ counts,  // kFellBack marks a serial-walk term
                                                          const uint32_t* __restrict__ cands,
                                                          ZgChunk* __restrict__ chunks, unsigned long long* err) {
  __shared__ uint32_t key[kCandCap];   // candidate offsets, sorted
  __shared__ uint32_t ul[kCandCap];    // uncompressed sizes
  __shared__ uint32_t cs[kCandCap];    // clen | scheme << 24 | kPointed | kGood
  __shared__ uint32_t nx[kCandCap];    // index of the successor candidate, kEnd or kNone
  __shared__ uint32_t part_n[kLinkThreads / kWave];
  __shared__ uint32_t part_u[kLinkThreads / kWave];
  __shared__ int ok;
  const int t = blockIdx.x;
  const ZgTerm tm = terms[t];
  const uint32_t n = counts[t];
  const int tid = threadIdx.x;
  // the fast path needs at least one candidate per planned chunk (terms of at most 4 GiB)
  if (n < tm.n_chunks || n == 0 || n > kCandCap || tm.src_len >= (uint64_t(1) << 32)) {
    if (tid == 0) {
      counts[t] = n | kFellBack;
      walk_term(tm, t, chunks, err, GlobalHdr{src + tm.src});
    }
    return;
  }
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t i = tid; i < P; i += kLinkThreads) key[i] = i < n ? cands[uint64_t(t) * kCandCap + i] : 0xFFFFFFFFu;
  if (tid == 0) ok = 1;
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {  // bitonic sort, ascending
    for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
      for (uint32_t i = tid; i < P; i += kLinkThreads) {
        const uint32_t l = i ^ jj;
        if (l > i) {
          const uint32_t a = key[i], b = key[l];
          if (((i & k) == 0) == (a > b)) {
            key[i] = b;
            key[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // successors
  const uint8_t* run = src + tm.src;
  for (uint32_t i = tid; i < n; i += kLinkThreads) {
    uint32_t lo, hi;
    load8(run + key[i], lo, hi);
    const uint32_t clen = lo >> 8;
    const uint64_t end = uint64_t(key[i]) + 8 + clen;
    nx[i] = end == tm.src_len ? kEnd : end < tm.src_len ? lds_find(key, n, uint32_t(end)) : kNone;
    ul[i] = hi >> 8;
    cs[i] = clen | (hi & 0xFF) << 24;
  }
  __syncthreads();
  for (uint32_t i = tid; i < n; i += kLinkThreads)
    if (nx[i] < n) atomicOr(&cs[nx[i]], kPointed);
  __syncthreads();
  for (uint32_t i = tid; i < n; i += kLinkThreads)
    if (nx[i] != kNone && (key[i] == 0 || (cs[i] & kPointed))) atomicOr(&cs[i], kGood);
  __syncthreads();
  for (uint32_t i = tid; i < n; i += kLinkThreads)  // closed under the successor
    if ((cs[i] & kGood) && nx[i] != kEnd && !(cs[nx[i]] & kGood)) ok = 0;
  if (tid == 0 && (key[0] != 0 || !(cs[0] & kGood))) ok = 0;
  // exclusive prefix sums (chunk count, uncompressed bytes) over the chain members: each thread
  // owns a contiguous slice, then a wave scan and the wave totals
  const uint32_t per = (n + kLinkThreads - 1) / kLinkThreads;
  const uint32_t a = min(n, tid * per), b = min(n, a + per);
  uint32_t cnt = 0, sum = 0;
  for (uint32_t i = a; i < b; ++i)
    if (cs[i] & kGood) {
      ++cnt;
      sum += ul[i];
    }
  uint32_t inc_n = cnt, inc_u = sum;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t yn = __shfl_up(inc_n, d, kWave), yu = __shfl_up(inc_u, d, kWave);
    if (int(lane_id()) >= d) {
      inc_n += yn;
      inc_u += yu;
    }
  }
  const int wv = tid / kWave;
  if (lane_id() == kWave - 1) {
    part_n[wv] = inc_n;
    part_u[wv] = inc_u;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t rn = 0, ru = 0;
    for (int k = 0; k < kLinkThreads / kWave; ++k) {
      const uint32_t xn = part_n[k], xu = part_u[k];
      part_n[k] = rn;
      part_u[k] = ru;
      rn += xn;
      ru += xu;
    }
    if (rn != tm.n_chunks || (tm.ulen != 0 && ru != tm.ulen)) ok = 0;
  }
  __syncthreads();
  if (!ok) {  // a broken or ambiguous chain: the serial walk decides
    if (tid == 0) {
      counts[t] = n | kFellBack;
      walk_term(tm, t, chunks, err, GlobalHdr{src + tm.src});
    }
    return;
  }
  uint32_t c = part_n[wv] + inc_n - cnt;  // this slice's first chunk index
  uint32_t off = part_u[wv] + inc_u - sum;
  for (uint32_t i = a; i < b; ++i) {
    if (!(cs[i] & kGood)) continue;
    ZgChunk ch;
    ch.src = tm.src + key[i] + 8;
    ch.dst = tm.dst + off;
    ch.clen = cs[i] & 0xFFFFFF;
    ch.ulen = ul[i];
    ch.scheme = (cs[i] >> 24) & 0x3F;
    ch.term = uint32_t(t);
    chunks[tm.chunk_base + c] = ch;
    ++c;
    off += ul[i];
  }
}

using zwv::wave_copy;  // wave64.h

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
// K3b: LZ4-frame (+BG4) decode.  One wave per chunk, 4 waves per 256-thread block, persistent
// grid.  Decoded bytes go through a small per-wave LDS history ring (4 KiB by default, so 8 waves
// per SIMD stay resident) and are flushed to HBM in 16-byte stores every 2 KiB.
//
//  * compressed stream: a 512-byte window held as two dwords per lane; token / length bytes are
//    read with v_readlane (uniform), literal bytes lane-parallel with ds_bpermute; the window
//    slides by 256 bytes so the next line's load overlaps the current line's parsing.
//  * lz4_fast takes the common short sequence (no length-extension bytes) with every check folded
//    into loop bounds and unconditional ring writes; the general path handles the rest.
//  * match copies: lane i of a 64-byte block reads source o - off*(1 + i/off) (the periodic form
//    of an overlapping copy, always a final byte); distances <= ring - 320 come from the LDS ring,
//    longer ones from HBM with L2-coherent loads (sc1, agent scope) after s_waitcnt vmcnt(0) --
//    those bytes were flushed by this wave at least ring - 320 - 2 KiB earlier.
//  * BG4: the grouped stream is scattered to its interleaved position (4*j + g) on flush, and
//    long-distance match reads use the same mapping, so no regroup pass or scratch is needed.
//  * chunks clipped by [clip_lo, clip_hi) decode into a 128 KiB slot of the caller's per-launch
//    scratch (one for the chunk straddling clip_lo, one for clip_hi), then the clipped range is
//    copied out.  The scratch belongs to the launch, so clipped decodes on several streams never
//    share it.
// --------------------------------------------------------------------------------------------
// Ring geometry (bytes per wave) is a template parameter RB: a larger ring keeps more match
// sources in LDS (fewer L2 read-backs) at the price of fewer resident waves per CU.
template <uint32_t RB> struct RingGeo {
  static constexpr uint32_t kMask = RB - 1;
  static constexpr uint32_t kReach = RB - 256 - 64;  // max match distance served from the ring
};
constexpr uint32_t kFlushAt = 2048;

constexpr uint32_t kClipSlot = kMaxChunk + 256;
static_assert(2 * kClipSlot == ZG_CLIP_SCRATCH_BYTES, "clip scratch layout");

using zgw::Win;
using zgw::load_u8_coherent;
using zgw::win_init;
using zgw::win_lane_u8;
using zgw::win_seek;
using zgw::win_u8;

// Optional decode profile (ZG_LZ4_PROF=1 selects the kProf instantiation).
__device__ unsigned long long g_lz4_prof[10];
__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

struct Sink {
  uint8_t* ring;  // this wave's LDS ring (16-byte aligned)
  uint8_t* out;   // chunk byte 0 in HBM (dst or scratch)
  uint32_t tmod;  // ring index of stream byte p = (tmod + p) & kRingMask
  uint32_t n;     // expected decoded size
  uint32_t op;    // bytes produced
  uint32_t fp;    // bytes flushed
  uint32_t g1, g2, g3;
  bool bg4;
  // profile counters (kProf only)
  uint64_t t_lit, t_match, t_flush, nseq, lit_bytes, match_bytes, nfar, nflush, nshort;
};

// Grouped-stream position -> byte offset in the chunk (identity unless BG4).
__device__ __forceinline__ uint32_t out_pos(const Sink& s, uint32_t p) {
  if (!s.bg4) return p;
  const uint32_t a1 = p >= s.g1, a2 = p >= s.g2, a3 = p >= s.g3;
  uint32_t base = 0;  // selects, not branches: the lanes of one flush straddle group boundaries
  base = a1 ? s.g1 : base;
  base = a2 ? s.g2 : base;
  base = a3 ? s.g3 : base;
  return 4 * (p - base) + a1 + a2 + a3;
}

template <uint32_t RB>
__device__ void sink_flush(Sink& s, uint32_t upto, bool final, uint32_t lane) {
  __builtin_amdgcn_wave_barrier();
  if (s.bg4) {
    for (uint32_t i = s.fp + lane; i < upto; i += kWave) s.out[out_pos(s, i)] = s.ring[(s.tmod + i) & RingGeo<RB>::kMask];
    s.fp = upto;
    return;
  }
  uint32_t p = s.fp;
  const uintptr_t a = reinterpret_cast<uintptr_t>(s.out) + p;
  uint32_t head = uint32_t((16 - (a & 15)) & 15);
  if (head > upto - p) head = upto - p;
  if (lane < head) s.out[p + lane] = s.ring[(s.tmod + p + lane) & RingGeo<RB>::kMask];
  p += head;
  const uint32_t nvec = (upto - p) >> 4;
  for (uint32_t v = lane; v < nvec; v += kWave) {
    const uint32_t q = p + 16 * v;
    const uint4 x = *reinterpret_cast<const uint4*>(s.ring + ((s.tmod + q) & RingGeo<RB>::kMask));
    *reinterpret_cast<uint4*>(s.out + q) = x;
  }
  p += 16 * nvec;
  if (final) {
    if (lane < upto - p) s.out[p + lane] = s.ring[(s.tmod + p + lane) & RingGeo<RB>::kMask];
    p = upto;
  }
  s.fp = p;
}

template <bool kProf, uint32_t RB>
__device__ __forceinline__ void sink_advance(Sink& s, uint32_t cnt, uint32_t lane) {
  s.op += cnt;
  if (s.op - s.fp >= kFlushAt) {
    const uint64_t t0 = kProf ? clk() : 0;
    sink_flush<RB>(s, s.op, false, lane);
    if (kProf) {
      s.t_flush += clk() - t0;
      s.nflush++;
    }
  }
}

// Copy `len` literal bytes starting at stream position a.
template <bool kProf, uint32_t RB>
__device__ __forceinline__ void copy_literals(Sink& s, Win& w, uint32_t a, uint32_t len, uint32_t lane) {
  for (uint32_t b = 0; b < len; b += kWave) {
    const uint32_t cnt = len - b < kWave ? len - b : kWave;
    win_seek(w, a + b, lane);
    const uint32_t v = win_lane_u8(w, a + b, lane);
    // unconditional: lanes past the literal write ring slots ahead of op (see lz4_fast)
    s.ring[(s.tmod + s.op + lane) & RingGeo<RB>::kMask] = uint8_t(v);
    sink_advance<kProf, RB>(s, cnt, lane);
  }
}

template <bool kProf, uint32_t RB>
__device__ __forceinline__ void copy_match(Sink& s, uint32_t off, uint32_t ml, uint32_t lane) {
  // lane i of each 64-byte block copies from distance back = off * (1 + i / off): the periodic form
  // of an overlapping copy, so every source byte is already final.
  uint32_t back = off;
  if (off < kWave) {
    const uint32_t magic = (65536u + off - 1) / off;  // exact floor(lane / off) for lane, off < 64
    back = off * (1 + ((lane * magic) >> 16));
  }
  if (off <= RingGeo<RB>::kReach) {
    for (uint32_t b = 0; b < ml; b += kWave) {
      const uint32_t cnt = ml - b < kWave ? ml - b : kWave;
      const uint32_t o = s.op + lane;
      __builtin_amdgcn_wave_barrier();
      if (lane < cnt) s.ring[(s.tmod + o) & RingGeo<RB>::kMask] = s.ring[(s.tmod + o - back) & RingGeo<RB>::kMask];
      sink_advance<kProf, RB>(s, cnt, lane);
    }
  } else {
    for (uint32_t b = 0; b < ml; b += kWave) {
      const uint32_t cnt = ml - b < kWave ? ml - b : kWave;
      const uint32_t o = s.op + lane;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane < cnt) s.ring[(s.tmod + o) & RingGeo<RB>::kMask] = uint8_t(load_u8_coherent(s.out + out_pos(s, o - back)));
      sink_advance<kProf, RB>(s, cnt, lane);
    }
  }
}

// Fast path for the common sequence shape of weight data: lit < 15 and ml < 19 (no length-
// extension bytes), a match source inside the LDS ring, >= 18 stream bytes left in the block.
// Measured (rocprofv3 PMC, BG4 bf16): the general path below is SALU-issue bound -- ~107 scalar
// instructions per sequence against one scalar unit per CU shared by ~20 waves -- so here every
// check is folded into two loop bounds (ip_lim: block end / stream window; op_lim: output room /
// next flush) and one offset range test, bytes come from one window gather (lane l = stream byte
// ip + l) plus read-lanes, and ring writes are unconditional: lanes past the sequence write into
// ring slots ahead of `op`, which are rewritten before they are flushed and lie more than
// RingGeo<RB>::kReach behind every later match source.  Returns at the first sequence it cannot take.
template <bool kProf, uint32_t RB>
__device__ __forceinline__ void lz4_fast(Sink& s, Win& w, uint32_t& ip, uint32_t end, uint32_t lane) {
  const uint32_t ip_end = end >= 18 ? end - 18 : 0;
  const uint32_t op_room = s.n >= 32 ? s.n - 32 : 0;
  while (true) {
    win_seek(w, ip, lane);
    const uint32_t ip_lim = ip_end < w.wofs + 256 ? ip_end : w.wofs + 256;
    if (ip >= ip_lim) return;
    uint32_t op_lim = op_room < s.fp + kFlushAt ? op_room : s.fp + kFlushAt;
    // One gather per sequence, aligned to its literals: lane l holds stream byte ip + 1 + l, so the
    // offset (lanes lit, lit + 1) and the NEXT token (lane lit + 2) are read-lanes of the same vector.
    uint32_t token = win_u8(w, ip);
    do {
      if (s.op >= op_lim) {
        if (s.op >= op_room) return;
        sink_flush<RB>(s, s.op, false, lane);
        op_lim = op_room < s.fp + kFlushAt ? op_room : s.fp + kFlushAt;
      }
      const uint32_t lit = token >> 4, mlc = token & 15;
      const uint32_t v = win_lane_u8(w, ip + 1, lane);
      const uint32_t off = __builtin_amdgcn_readlane(v, int(lit)) | (__builtin_amdgcn_readlane(v, int(lit + 1)) << 8);
      const uint32_t next = __builtin_amdgcn_readlane(v, int(lit + 2));
      // one exit test: a length-extension nibble, or an offset of 0 / before the chunk start (the
      // general path then decodes the sequence, or reports it)
      if (uint32_t(lit == 15) | uint32_t(mlc == 15) | uint32_t(off - 1 >= s.op + lit)) return;
      s.ring[(s.tmod + s.op + lane) & RingGeo<RB>::kMask] = uint8_t(v);
      const uint32_t mo = s.op + lit;
      uint8_t m;
      if (off <= RingGeo<RB>::kReach) {
        uint32_t back = off;
        if (off < kWave) back = off * (1 + ((lane * ((65536u + off - 1) / off)) >> 16));
        __builtin_amdgcn_wave_barrier();
        m = s.ring[(s.tmod + mo + lane - back) & RingGeo<RB>::kMask];
      } else {
        // Far match (off > ring reach >= 64, so no overlap): the source was flushed at least
        // reach - kFlushAt bytes ago; wait for this wave's stores, then read it back through L2.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        m = uint8_t(load_u8_coherent(s.out + out_pos(s, mo + lane - off)));
        if (kProf) s.nfar++;
      }
      __builtin_amdgcn_wave_barrier();
      s.ring[(s.tmod + mo + lane) & RingGeo<RB>::kMask] = m;
      __builtin_amdgcn_wave_barrier();
      if (kProf) {
        s.nseq++;
        s.lit_bytes += lit;
        s.match_bytes += mlc + 4;
        s.nshort += off < kWave;
      }
      s.op = mo + mlc + 4;
      ip += lit + 3;
      token = next;
    } while (ip < ip_lim);
  }
}

// One LZ4 block at stream positions [blk, blk + blen). Returns false on malformed input.
template <bool kProf, uint32_t RB>
__device__ bool lz4_block(Sink& s, Win& w, uint32_t blk, uint32_t blen, uint32_t lane) {
  const uint32_t end = blk + blen;
  uint32_t ip = blk;
  while (true) {
    if (ip >= end) return false;
    lz4_fast<kProf, RB>(s, w, ip, end, lane);
    win_seek(w, ip, lane);
    const uint32_t token = win_u8(w, ip);
    ++ip;
    uint32_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= end) return false;
        win_seek(w, ip, lane);
        b = win_u8(w, ip);
        ++ip;
        lit += b;
      } while (b == 255);
    }
    if (lit > end - ip || lit > s.n - s.op) return false;
    if (kProf) s.nseq++;
    if (lit) {
      const uint64_t t0 = kProf ? clk() : 0;
      copy_literals<kProf, RB>(s, w, ip, lit, lane);
      if (kProf) {
        s.t_lit += clk() - t0;
        s.lit_bytes += lit;
      }
    }
    ip += lit;
    if (ip == end) return true;  // last sequence: literals only
    if (end - ip < 2) return false;
    win_seek(w, ip, lane);
    const uint32_t off = win_u8(w, ip) | (win_u8(w, ip + 1) << 8);
    ip += 2;
    if (off == 0 || off > s.op) return false;
    uint32_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (ip >= end) return false;
        win_seek(w, ip, lane);
        b = win_u8(w, ip);
        ++ip;
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (ml > s.n - s.op) return false;
    const uint64_t t0 = kProf ? clk() : 0;
    copy_match<kProf, RB>(s, off, ml, lane);
    if (kProf) {
      s.t_match += clk() - t0;
      s.match_bytes += ml;
      s.nfar += off > RingGeo<RB>::kReach;
      s.nshort += off < kWave;
    }
  }
}

// Decode an LZ4 frame of clen bytes; returns false on malformed input.
template <bool kProf, uint32_t RB>
__device__ bool lz4_frame(Sink& s, const uint8_t* payload, uint32_t clen, uint32_t lane) {
  Win w;
  win_init(w, payload, lane);
  const uint32_t k = uint32_t(reinterpret_cast<uintptr_t>(payload) & 3);  // stream pos = k + byte index
  if (clen < 7) return false;
  const uint32_t magic = win_u8(w, k) | (win_u8(w, k + 1) << 8) | (win_u8(w, k + 2) << 16) | (win_u8(w, k + 3) << 24);
  if (magic != 0x184D2204u) return false;
  const uint32_t flg = win_u8(w, k + 4);
  if ((flg >> 6) != 1) return false;
  uint32_t ip = 7 + ((flg & 8) ? 8 : 0) + ((flg & 1) ? 4 : 0);
  const bool block_ck = flg & 0x10;
  while (true) {
    if (ip > clen || clen - ip < 4) return false;
    win_seek(w, k + ip, lane);
    const uint32_t bs = win_u8(w, k + ip) | (win_u8(w, k + ip + 1) << 8) | (win_u8(w, k + ip + 2) << 16) |
                        (win_u8(w, k + ip + 3) << 24);
    ip += 4;
    if (bs == 0) return true;
    const uint32_t len = bs & 0x7FFFFFFFu;
    if (len > clen - ip) return false;
    if (bs & 0x80000000u) {
      if (len > s.n - s.op) return false;
      copy_literals<kProf, RB>(s, w, k + ip, len, lane);
    } else if (!lz4_block<kProf, RB>(s, w, k + ip, len, lane)) {
      return false;
    }
    ip += len + (block_ck ? 4 : 0);
  }
}

template <bool kProf, uint32_t RB>
__global__ void __launch_bounds__(256, RB <= 4096 ? 8 : 5) k_decode_lz4(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                    const ZgChunk* __restrict__ chunks, int n_chunks,
                                                    uint64_t clip_lo, uint64_t clip_hi, uint8_t* __restrict__ clip_scratch,
                                                    unsigned long long* err, uint64_t src_n, uint64_t dst_n) {
  __shared__ __attribute__((aligned(16))) uint8_t rings[kWavesPerBlock][RB];
  const uint32_t lane = lane_id();
  const int wave = wave_uniform(int(threadIdx.x >> 6));
  const int stride = int(gridDim.x) * kWavesPerBlock;
  uint64_t prof[10] = {};
  for (int c = wave_uniform(int(blockIdx.x) * kWavesPerBlock + wave); c < n_chunks; c += stride) {
    const ZgChunk ch = chunks[c];
    if (ch.scheme == 0) continue;
    if (ch.src + ch.clen > src_n || ch.dst + ch.ulen > dst_n) {
      if (lane == 0) report(err, ZG_ERR_RANGE, uint32_t(c));
      continue;
    }
    if (ch.ulen > kMaxChunk) {
      if (lane == 0) report(err, ZG_ERR_CAPACITY, uint32_t(c));
      continue;
    }
    const uint64_t end = ch.dst + ch.ulen;
    const uint64_t lo = ch.dst > clip_lo ? ch.dst : clip_lo;
    const uint64_t hi = end < clip_hi ? end : clip_hi;
    if (lo >= hi) continue;
    const bool clipped = lo != ch.dst || hi != end;
    const uint64_t t_start = kProf ? clk() : 0;
    Sink s{};
    s.ring = rings[wave];
    s.out = clipped ? clip_scratch + (ch.dst < clip_lo ? 0u : kClipSlot) : dst + ch.dst;
    s.bg4 = ch.scheme == 2;
    s.tmod = s.bg4 ? 0u : uint32_t(reinterpret_cast<uintptr_t>(s.out) & RingGeo<RB>::kMask);
    s.n = ch.ulen;
    const uint32_t q = ch.ulen >> 2, r = ch.ulen & 3;
    s.g1 = q + (r > 0 ? 1u : 0u);
    s.g2 = s.g1 + q + (r > 1 ? 1u : 0u);
    s.g3 = s.g2 + q + (r > 2 ? 1u : 0u);
    const bool ok = lz4_frame<kProf, RB>(s, src + ch.src, ch.clen, lane);
    if (!ok) {
      if (lane == 0) report(err, ZG_ERR_LZ4, uint32_t(c));
      continue;
    }
    if (s.op != ch.ulen) {
      if (lane == 0) report(err, ZG_ERR_SIZE, uint32_t(c));
      continue;
    }
    sink_flush<RB>(s, s.op, true, lane);
    if (kProf) {
      const uint64_t v[10] = {s.t_lit, s.t_match, s.t_flush, clk() - t_start, s.nseq,
                              s.lit_bytes, s.match_bytes, s.nfar, s.nflush, s.nshort};
      for (int i = 0; i < 10; ++i) prof[i] += v[i];
    }
    if (clipped) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t a = uint32_t(lo - ch.dst), len = uint32_t(hi - lo);
      for (uint32_t i = lane; i < len; i += kWave) dst[lo + i] = uint8_t(load_u8_coherent(s.out + a + i));
    }
  }
  if (kProf && lane == 0)
    for (int i = 0; i < 10; ++i) atomicAdd(&g_lz4_prof[i], (unsigned long long)prof[i]);
}

// --------------------------------------------------------------------------------------------
// K1: keyed BLAKE3 chunk hashes, latency path (launches without scratch; the leaf-flat pipeline
// in blake3_flat.hip is the throughput path).  One wave per Xet chunk (4 per 256-thread block);
// lane l owns BLAKE3 chunks l, l+64 (<= 128 for a 128 KiB Xet chunk); chaining values are merged
// pairwise in LDS (pairwise-with-carry == BLAKE3's left-complete tree).
// --------------------------------------------------------------------------------------------
using zg::store_hash;
using zg::wave_hash;

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

size_t zg_index_scratch_bytes(int n_terms) {
  return (size_t(n_terms) * 4 + 255) / 256 * 256 + size_t(n_terms) * kCandCap * 4;
}

hipError_t zg_index_terms_scan(const uint8_t* src, uint64_t src_n, const ZgTerm* terms, int n_terms, ZgChunk* chunks,
                               unsigned long long* err, uint8_t* scratch, size_t scratch_bytes, hipStream_t stream) {
  if (n_terms <= 0) return hipSuccess;
  if (scratch == nullptr || scratch_bytes < zg_index_scratch_bytes(n_terms) || (reinterpret_cast<uintptr_t>(src) & 15))
    return zg_index_terms(src, terms, n_terms, chunks, err, stream);
  uint32_t* counts = reinterpret_cast<uint32_t*>(scratch);
  uint32_t* cands = reinterpret_cast<uint32_t*>(scratch + (size_t(n_terms) * 4 + 255) / 256 * 256);
  hipError_t e = hipMemsetAsync(counts, 0, size_t(n_terms) * 4, stream);
  if (e != hipSuccess) return e;
  const uint64_t per_block = uint64_t(kScanThreads) * kScanBytesPerThread;
  const uint64_t blocks = (src_n + per_block - 1) / per_block;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_hdr_scan, dim3(uint32_t(blocks ? blocks : 1)), dim3(kScanThreads), 0, stream, src, src_n, terms,
                     n_terms, counts, cands);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_hdr_link, dim3(n_terms), dim3(kLinkThreads), 0, stream, src, terms, counts, cands, chunks, err);
  return hipGetLastError();
}

hipError_t zg_place_chunks(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                           int n_chunks, uint64_t clip_lo, uint64_t clip_hi, uint8_t* clip_scratch,
                           unsigned long long* err, hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  const bool clipped = clip_lo > 0 || clip_hi < dst_n;
  if (clipped && clip_scratch == nullptr) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_place_raw, dim3((n_chunks + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, stream, src,
                     dst, chunks, n_chunks, clip_lo, clip_hi, src_n, dst_n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // ZG_LZ4_SEQ=0 forces the LDS-ring decoder (A/B runs); clip windows always use it.
  static const bool batched = [] {
    const char* v = getenv("ZG_LZ4_SEQ");
    return !(v && *v == '0');
  }();
  if (batched && !clipped) return zg_lz4_batched_decode(src, src_n, dst, dst_n, chunks, n_chunks, err, stream);
  const int blocks = (n_chunks + kWavesPerBlock - 1) / kWavesPerBlock;
  // ZG_LZ4_GRID caps the persistent grid (occupancy experiments: 256 = one wave per SIMD).
  static const int grid_cap = [] {
    const char* v = getenv("ZG_LZ4_GRID");
    const int g = v ? atoi(v) : 0;
    return g > 0 && g < 1280 ? g : 1280;
  }();
  static const bool prof = [] {
    const char* v = getenv("ZG_LZ4_PROF");
    return v && *v && *v != '0';
  }();
  // ZG_LZ4_RING = ring KiB per wave (4, 8, 16 or 32); resident blocks per CU follow from the LDS.
  // Measured on BG4 bf16 (1 GiB, 16.7k chunks): 4 KiB 46.3 GB/s (8 waves/SIMD, more matches read
  // back from L2), 8 KiB 38.2, 16 KiB 29.9, 32 KiB 18.5 -- occupancy beats ring reach.
  static const int ring_kib = [] {
    const char* v = getenv("ZG_LZ4_RING");
    const int k = v ? atoi(v) : 4;
    return k == 8 || k == 16 || k == 32 ? k : 4;
  }();
  const int per_cu = ring_kib == 4 ? 8 : ring_kib == 8 ? 5 : ring_kib == 16 ? 2 : 1;
  const int cap = grid_cap < 256 * per_cu ? grid_cap : 256 * per_cu;
  const int grid = blocks < cap ? blocks : cap;
  if (prof) {
    unsigned long long zero[10] = {};
    hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lz4_prof), zero, sizeof zero, 0, hipMemcpyHostToDevice, stream);
  }
#define ZG_LZ4_LAUNCH(P, R)                                                                                       \
  hipLaunchKernelGGL((k_decode_lz4<P, R>), dim3(grid), dim3(256), 0, stream, src, dst, chunks, n_chunks, clip_lo, \
                     clip_hi, clip_scratch, err, src_n, dst_n)
  if (ring_kib == 4) {
    if (prof) ZG_LZ4_LAUNCH(true, 4096); else ZG_LZ4_LAUNCH(false, 4096);
  } else if (ring_kib == 16) {
    if (prof) ZG_LZ4_LAUNCH(true, 16384); else ZG_LZ4_LAUNCH(false, 16384);
  } else if (ring_kib == 32) {
    if (prof) ZG_LZ4_LAUNCH(true, 32768); else ZG_LZ4_LAUNCH(false, 32768);
  } else {
    if (prof) ZG_LZ4_LAUNCH(true, 8192); else ZG_LZ4_LAUNCH(false, 8192);
  }
#undef ZG_LZ4_LAUNCH
  if (prof) {
    unsigned long long v[10];
    hipMemcpyFromSymbolAsync(v, HIP_SYMBOL(g_lz4_prof), sizeof v, 0, hipMemcpyDeviceToHost, stream);
    hipStreamSynchronize(stream);
    if (v[4])
      fprintf(stderr,
              "{\"lz4_prof\": {\"chunks\": %d, \"t_lit\": %llu, \"t_match\": %llu, \"t_flush\": %llu, \"t_total\": %llu, "
              "\"nseq\": %llu, \"lit_bytes\": %llu, \"match_bytes\": %llu, \"nfar\": %llu, \"nflush\": %llu, "
              "\"nshort\": %llu}}\n",
              n_chunks, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9]);
  }
  return hipGetLastError();
}

hipError_t zg_hash_chunks(const uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks, int n_chunks, uint8_t* hashes,
                          uint64_t* sizes, uint32_t hash_index_base, uint8_t* scratch, size_t scratch_bytes,
                          hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  if (scratch)
    return zg_hash_chunks_flat(dst, dst_n, chunks, n_chunks, hashes + 32 * uint64_t(hash_index_base),
                               sizes ? sizes + hash_index_base : nullptr, scratch, scratch_bytes, stream);
  hipLaunchKernelGGL(k_hash_chunks, dim3((n_chunks + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, stream, dst,
                     chunks, n_chunks, hashes, sizes, hash_index_base, dst_n);
  return hipGetLastError();
}

hipError_t zg_ingest_chunks(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                            int n_chunks, int has_compressed, unsigned long long* err, uint8_t* hashes,
                            uint64_t* sizes, uint32_t hash_index_base, uint8_t* scratch, size_t scratch_bytes,
                            hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  if (!scratch) return hipErrorInvalidValue;
  uint8_t* h = hashes + 32 * uint64_t(hash_index_base);
  uint64_t* sz = sizes ? sizes + hash_index_base : nullptr;
  int hashed = 0;  // the decoder hashed the compressed chunks itself (zg_lz4_decode_ingest)
  if (has_compressed) {
    // the hash scratch doubles as the BG4 staging of the decoder (which finishes before the place/hash
    // pass below uses it: one stream); zg_ingest_scratch_bytes sizes it for both
    const hipError_t e = zg_lz4_decode_ingest(src, src_n, dst, dst_n, chunks, n_chunks, err, h, sz, &hashed, scratch,
                                              scratch_bytes, stream);
    if (e != hipSuccess) return e;
  }
  if (hashed)
    return zg_place_hash_flat_raw(src, src_n, dst, dst_n, chunks, n_chunks, err, h, sz, scratch, scratch_bytes, stream);
  return zg_place_hash_flat(src, src_n, dst, dst_n, chunks, n_chunks, err, h, sz, scratch, scratch_bytes, stream);
}

hipError_t zg_hash_ranges(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lens, int n, uint8_t* hashes,
                          int key_mode, uint8_t* scratch, size_t scratch_bytes, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (scratch) return zg_hash_ranges_flat(buf, offsets, lens, n, hashes, key_mode, scratch, scratch_bytes, stream);
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
