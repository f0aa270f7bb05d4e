// K3c: batched LZ4 / BG4-LZ4 decode for gfx950 (CDNA4, wave64).
//
// Xet weight chunks decode into ~6.8k LZ4 sequences per 64 KiB (BG4 bf16: the exponent planes
// are almost all 4-5 byte matches).  The LDS-ring decoder (k_decode_lz4, ingest.hip) executes
// those sequences one at a time with the whole wave, so ~5 of 64 lanes do useful work and every
// sequence pays a chain of read-lanes, LDS round trips and barriers (PMC: ~450 SIMD cycles per
// sequence).  This decoder keeps one wave per chunk (full occupancy) but splits LZ4's sequential
// and parallel halves:
//
//   parse    the token stream is walked with uniform (scalar) control flow, reading bytes from a
//            wave-wide register window; each sequence becomes one record {gap, literal length,
//            match length, offset} written into lane n of two VGPRs (a lane select) -- no memory.
//   execute  every 64 records: DPP prefix sums give each record's literal source and output
//            position; literal bytes, then match bytes, are produced one per lane per pass (the
//            lane -> record map is a scatter of record heads into LDS + a DPP max-scan).  A match
//            byte reads its periodic source (start - off + k mod off, always before the match);
//            when that byte is written by another lane of the same pass, the lane follows that
//            lane's source (pointer chase, almost never taken: it is skipped unless some source
//            lies at or after the pass's first destination).  Output goes straight to HBM, read
//            back through L2 after s_waitcnt vmcnt(0); BG4 chunks are scattered to their
//            interleaved byte (4 j + group) on store.
//
// Lengths/offsets are validated in the execute step (lane-parallel) before any byte moves.
// Clipped launches keep using the LDS-ring decoder.  Host oracle: csrc/core/lz4.cpp, compared
// bit-exactly in tests/test_gpu_kernels.py.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "blake3_dev.h"
#include "lz4win.h"
#include "wave64.h"
#include "zgpu.h"

namespace {

using zgw::Win;
using zgw::load_u8_coherent;
using zgw::win_init;
using zgw::win_lane_u8;
using zgw::win_seek;
using zgw::win_u8;
using zwv::scan_add;
using zwv::scan_max;

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr uint32_t kMaxChunk = 128u * 1024u;
constexpr uint32_t kMaxRecsPerSeq = 8;  // 1 + 2 literal splits + 4 match splits (<= 128 KiB), + 1 spare
constexpr uint32_t kFlushAbove = kWave - kMaxRecsPerSeq;
constexpr uint32_t kRing = 4096;  // LDS history per wave (power of two): 8 waves / SIMD stay resident

__device__ __forceinline__ void report(unsigned long long* err, uint32_t code, uint32_t idx) {
  if (err) atomicCAS(err, 0ull, (static_cast<unsigned long long>(code) << 32) | idx);
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return uint64_t(uni(uint32_t(v))) | (uint64_t(uni(uint32_t(v >> 32))) << 32);
}

__device__ __forceinline__ uint32_t shfl(uint32_t v, uint32_t lane) {
  return uint32_t(__builtin_amdgcn_ds_bpermute(int(lane << 2), int(v)));
}


// Smallest lane s with a[s] >= t (a non-decreasing over lanes); 64 if none.
__device__ __forceinline__ uint32_t find_ge(uint32_t a, uint32_t t) {
  uint32_t j = 0;
#pragma unroll
  for (uint32_t step = 32; step; step >>= 1) {
    const uint32_t v = shfl(a, j + step - 1);
    j += v < t ? step : 0u;
  }
  return j;
}

// k mod o for k < 2^16, 1 <= o < 2^16 (float reciprocal estimate + one correction).
__device__ __forceinline__ uint32_t umod16(uint32_t k, uint32_t o) {
  const int q = int(float(k) * __builtin_amdgcn_rcpf(float(o)));
  int r = int(k) - q * int(o);
  r += r < 0 ? int(o) : 0;
  r -= r >= int(o) ? int(o) : 0;
  return uint32_t(r);
}

struct Ctx {
  const uint8_t* pay;  // chunk payload (LZ4 frame)
  uint8_t* out;        // chunk output
  uint32_t clen, ulen;
  bool bg4;
  uint32_t g1, g2, g3;  // BG4 group starts in the grouped stream
  uint32_t k0;          // payload address & 3: stream position = k0 + payload byte index
  uint32_t obase;       // output (grouped) offset of the next batch
  uint32_t* heads;      // this wave's 64-entry LDS scratch
  uint8_t* ring;        // this wave's kRing-byte LDS history of recent output
  uint32_t* pf = nullptr;  // 64-dword LDS sink of the parse's stream prefetch (nullptr: none)
};

// Grouped-stream position -> byte offset in the chunk (identity unless BG4).
__device__ __forceinline__ uint32_t bmap(const Ctx& X, uint32_t p) {
  if (!X.bg4) return p;
  // grouped position p of group g (start G_g) lands at 4 (p - G_g) + g = 4 p + (g - 4 G_g): one
  // per-group constant, picked by the three group-start compares
  uint32_t c = p >= X.g1 ? 1u - 4u * X.g1 : 0u;
  c = p >= X.g2 ? 2u - 4u * X.g2 : c;
  c = p >= X.g3 ? 3u - 4u * X.g3 : c;
  return 4u * p + c;
}

// Records of the current batch: lane i holds record i (rl = gap | lit << 16, rh = ml | off << 16).
// Record formats (per lane), chosen so the common sequence costs the parse almost nothing:
//   short (fast path): rl = literal stream position, rh = the 4 stream bytes after the literals
//                      (offset in the low 16 bits), rx = 0; exec_batch loads the token byte
//                      before the literals
//   general:           rl = literal stream position, rh = offset, rx = 1 << 31 | ml << 16 | lit
//                      (lit <= 0xFFFF, ml <= 0x7FFF after splitting)
// Stream positions are relative to the dword-aligned payload base (k0 + byte index).
struct Batch {
  uint32_t rl, rh, rx;  // per lane
  uint32_t n;           // uniform: records held
};

// Lane -> index of the record whose [excl, incl) byte range covers byte t0 + lane: records that
// intersect the pass write their index at their first byte in the pass (unique), then a max-scan.
__device__ __forceinline__ uint32_t owner(const Ctx& X, uint32_t excl, uint32_t incl, uint32_t t0, uint32_t lane) {
  X.heads[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (incl > excl && excl < t0 + kWave && incl > t0) X.heads[excl > t0 ? excl - t0 : 0] = lane;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const uint32_t h = X.heads[lane];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return scan_max(h);
}

// One match pass: lane -> (destination d, resolved source q) for match bytes t0 .. t0 + 63.
struct MatchLane {
  uint32_t d, q;
  bool on;
};

__device__ __forceinline__ MatchLane match_pass(const Ctx& X, uint32_t mi, uint32_t ml, uint32_t mstart, uint32_t off,
                                                uint32_t mtot, uint32_t t0, uint32_t lane) {
  MatchLane m;
  const uint32_t t = t0 + lane;
  m.on = t < mtot;
  const uint32_t s = owner(X, mi - ml, mi, t0, lane);
  const uint32_t k = t - shfl(mi - ml, s);
  const uint32_t st = shfl(mstart, s);
  uint32_t o = shfl(off, s);
  o = o ? o : 1u;
  m.d = m.on ? st + k : 0xFFFFFFFFu;
  m.q = m.on ? st - o + umod16(k, o) : 0u;  // periodic source, before the match start
  const uint32_t dfirst = uni(m.d);           // lane 0 is always on
  if (__builtin_amdgcn_ballot_w64(m.on && m.q >= dfirst)) {
    while (true) {  // sources written by this same pass: take the writer's source instead
      uint32_t j = find_ge(m.d, m.q);
      j = j > 63 ? 63 : j;
      const bool pend = m.on && shfl(m.d, j) == m.q;
      if (!__builtin_amdgcn_ballot_w64(pend)) break;
      const uint32_t qj = shfl(m.q, j);
      m.q = pend ? qj : m.q;
    }
  }
  return m;
}

// One wait for a pass group's four loads, stated as an asm that redefines the values: the stores
// that follow then carry no pending-load dependence.  Without it the compiler, unable to track the
// loads through the divergent pass branches, puts s_waitcnt vmcnt(0) before every byte store, and
// since vmcnt also counts stores, each store waited for the previous store's write acknowledgement.
// Measured (profiles/lz4_records_r3.md): far-match data +5 %, BG4 bf16 unchanged (the batched
// decoder is bound by its scalar parse, not by these waits).
__device__ __forceinline__ void land4(uint32_t v[4]) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) : : "memory");
}

// Output byte -> LDS history ring (recent output, for near match sources) and HBM.
__device__ __forceinline__ void put_byte(const Ctx& X, uint32_t p, uint32_t v) {
  X.ring[p & (kRing - 1)] = uint8_t(v);
  X.out[bmap(X, p)] = uint8_t(v);
}

// Literal runs of at least kWideLit bytes in a long batch (BG4 bf16: the two mantissa planes of a
// chunk are ~16 KiB literal runs each, ~half of every chunk's output) are copied 1 KiB per wave
// step: lane i moves stream bytes i, i + 64, ..., i + 960, sixteen byte loads then sixteen byte
// stores from one address each with immediate offsets (64 B apart in the payload; 256 B apart in a
// BG4 group's output, 64 B otherwise).  Every load and store instruction stays coalesced (64
// consecutive payload bytes; 64 output bytes 4 apart = 4 lines), and the lane -> record map,
// shuffles and BG4 address math of the lane-per-byte literal passes (~35 wave instructions per 64
// bytes) drop to ~2.  (A 16-bytes-per-lane variant -- one dwordx4-sized read per lane -- scattered
// each byte store over 64 lines and made the one-wave decoder 10 % slower.)  Only long batches take
// it: their match sources come back from HBM and their LDS ring is rebuilt from HBM afterwards, so
// these bytes need not enter the ring.
constexpr uint32_t kWideLit = 512;

__device__ __forceinline__ void wide_literals(const Ctx& X, uint32_t src, uint32_t dst, uint32_t n, uint32_t lane) {
  constexpr uint32_t kStep = 16 * kWave;
  uint32_t base = 0;
  for (; base + kStep <= n; base += kStep) {
    const uint8_t* a = X.pay + src + base + lane;
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = a[j * kWave];
    const uint32_t q0 = bmap(X, dst + base), q1 = bmap(X, dst + base + kStep - 1);
    if (!X.bg4) {
      uint8_t* o = X.out + q0 + lane;
#pragma unroll
      for (int j = 0; j < 16; ++j) o[j * kWave] = uint8_t(v[j]);
    } else if (q1 - q0 == 4 * (kStep - 1)) {  // one BG4 group: byte p goes to 4 p + c
      uint8_t* o = X.out + q0 + 4 * lane;
#pragma unroll
      for (int j = 0; j < 16; ++j) o[j * 4 * kWave] = uint8_t(v[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) X.out[bmap(X, dst + base + uint32_t(j) * kWave + lane)] = uint8_t(v[j]);
    }
  }
  for (uint32_t p = base + lane; p < n; p += kWave) X.out[bmap(X, dst + p)] = X.pay[src + p];
}

// Execute the batch's records.  Returns false (nothing written for the bad records) when any
// record is out of range.
//
// Sources: a byte less than kRing behind the batch's last output byte is still in this wave's LDS
// ring (nothing newer has wrapped onto its slot, and a short batch writes no two bytes kRing
// apart); older ("far") bytes come from HBM through L2.
// All far bytes of a short batch precede the batch, and the s_waitcnt at batch start has made
// every earlier store visible, so up to four passes' far loads are issued together and no pass
// waits on a store.  A long batch (a long literal run) can have far sources inside itself: its
// passes run one at a time, each after s_waitcnt vmcnt(0).
__device__ bool exec_batch(Batch& B, Ctx& X, uint32_t lane) {
  const bool valid = lane < B.n;
  const bool gen = (B.rx >> 31) != 0;
  // short records carry only the literals' stream position (the parse spends no scalar work on
  // packing the token): the token byte just before them is loaded here, lane-parallel, per batch
  const uint32_t lpos = B.rl - X.k0;  // payload offset of this record's literals
  const uint32_t tok = valid && !gen ? uint32_t(X.pay[lpos - 1 < X.clen ? lpos - 1 : 0u]) : 0u;
  const uint32_t lit = !valid ? 0u : gen ? (B.rx & 0xFFFF) : tok >> 4;
  const uint32_t ml = !valid ? 0u : gen ? ((B.rx >> 16) & 0x7FFF) : (tok & 15) + 4;
  const uint32_t off = B.rh & 0xFFFF;
  const uint32_t a2 = scan_add(lit + ml);
  const uint32_t span = __builtin_amdgcn_readlane(a2, 63);
  const bool long_batch = span + 4 * kWave >= kRing;
  // long literal runs of a long batch go through wide_literals, the rest one byte per lane
  const bool wide = long_batch && lit >= kWideLit;
  const uint32_t litp = wide ? 0u : lit;
  const uint32_t li = scan_add(litp), mi = scan_add(ml);
  const uint32_t opos = X.obase + a2 - lit - ml;  // output offset of the record
  const uint32_t mstart = opos + lit;          // output offset of its match
  const bool bad = valid && (lpos + lit > X.clen || mstart + ml > X.ulen || (ml && (off == 0 || off > mstart)));
  B.n = 0;
  B.rl = B.rh = B.rx = 0;
  if (__builtin_amdgcn_ballot_w64(bad)) return false;
  const uint32_t ltot = __builtin_amdgcn_readlane(li, 63), mtot = __builtin_amdgcn_readlane(mi, 63);
  X.obase += span;
  const uint32_t oend = X.obase;  // one past the batch's last output byte
  // Far match sources (kRing or more behind the batch end) are read back from HBM, so every earlier
  // store must be acknowledged first; a short batch whose sources all lie in the LDS ring skips
  // that wait (BG4 exponent-plane matches are short-range).
  if (long_batch || __builtin_amdgcn_ballot_w64(ml != 0 && oend - (mstart - off) >= kRing))
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // earlier batches' stores are in L2
  for (uint64_t wm = __builtin_amdgcn_ballot_w64(wide); wm; wm &= wm - 1) {
    const uint32_t r = uint32_t(__builtin_ctzll(wm));
    wide_literals(X, __builtin_amdgcn_readlane(lpos, r), __builtin_amdgcn_readlane(opos, r),
                  __builtin_amdgcn_readlane(lit, r), lane);
  }
  // literal bytes, one per lane; four passes' loads in flight at once
  for (uint32_t g0 = 0; g0 < ltot; g0 += 4 * kWave) {
    uint32_t to[4], v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t t0 = g0 + uint32_t(j) * kWave;
      to[j] = 0xFFFFFFFFu;
      v[j] = 0;
      if (t0 < ltot) {
        const uint32_t t = t0 + lane;
        const uint32_t s = owner(X, li - litp, li, t0, lane);
        const uint32_t k = t - shfl(li - litp, s);
        const uint32_t from = shfl(lpos, s) + k, dst = shfl(opos, s) + k;  // all lanes shuffle
        if (t < ltot) {
          to[j] = dst;
          v[j] = X.pay[from];
        }
      }
    }
    land4(v);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (to[j] != 0xFFFFFFFFu) put_byte(X, to[j], v[j]);
  }
  if (!long_batch) {
    // short batch: far sources all precede it (already visible); group four passes
    for (uint32_t g0 = 0; g0 < mtot; g0 += 4 * kWave) {
      MatchLane m[4];
      uint32_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t t0 = g0 + uint32_t(j) * kWave;
        m[j].on = false;
        v[j] = 0;
        if (t0 < mtot) {
          m[j] = match_pass(X, mi, ml, mstart, off, mtot, t0, lane);
          if (m[j].on && oend - m[j].q >= kRing) v[j] = load_u8_coherent(X.out + bmap(X, m[j].q));
        }
      }
      land4(v);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!m[j].on) continue;
        const uint32_t x = oend - m[j].q >= kRing ? v[j] : uint32_t(X.ring[m[j].q & (kRing - 1)]);
        put_byte(X, m[j].d, x);
      }
    }
  } else {
    // Long batch: its literal phase wrote bytes kRing or more apart out of position order (a
    // literal can be overwritten in the ring by an earlier match byte kRing before it), so the
    // ring is not trusted here: every source is read back from HBM, one pass at a time, and the
    // ring is rebuilt from HBM afterwards.
    for (uint32_t t0 = 0; t0 < mtot; t0 += kWave) {
      const MatchLane m = match_pass(X, mi, ml, mstart, off, mtot, t0, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this batch's earlier stores are in L2
      if (m.on) X.out[bmap(X, m.d)] = uint8_t(load_u8_coherent(X.out + bmap(X, m.q)));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ring rebuild: eight loads per lane in flight before their LDS stores (one L2 round trip per
    // 512 bytes instead of one per 64)
    const uint32_t lo = oend > kRing ? oend - kRing : 0u;
    for (uint32_t p0 = lo; p0 < oend; p0 += 8 * kWave) {
      uint32_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t p = p0 + uint32_t(j) * kWave + lane;
        v[j] = p < oend ? load_u8_coherent(X.out + bmap(X, p)) : 0u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t p = p0 + uint32_t(j) * kWave + lane;
        if (p < oend) X.ring[p & (kRing - 1)] = uint8_t(v[j]);
      }
    }
  }
  return true;
}

// Append one LZ4 sequence (literal run at stream position lp) as general records; literal runs
// are split at 0xFFFF and matches at 0x7FFF (a split match keeps its offset, exact for LZ4's
// byte-sequential copy).  A chunk is <= 128 KiB, so one call adds at most kMaxRecsPerSeq records; the
// caller executes the batch before it could overflow.
__device__ __forceinline__ void emit(Batch& B, uint32_t lane, uint32_t lp, uint32_t lit, uint32_t ml, uint32_t off) {
  do {
    const uint32_t l = lit > 0xFFFFu ? 0xFFFFu : lit;
    const uint32_t m = lit > 0xFFFFu ? 0u : (ml > 0x7FFFu ? 0x7FFFu : ml);
    const bool me = lane == B.n;  // the lane that holds this record
    B.rl = me ? lp : B.rl;
    B.rh = me ? off : B.rh;
    B.rx = me ? 0x80000000u | (m << 16) | l : B.rx;
    ++B.n;
    lp += l;
    lit -= l;
    ml -= m;
  } while (lit | ml);
}

// Stream reader for the (wave-uniform) parse: 8 bytes at stream position p through a scalar
// load (s_load_dwordx2 at the dword below p: a scalar load ignores the two low bits of its byte
// offset, so p goes in as it is -- one scalar instruction less per sequence on the parse's chain).  The compressed payload is read-only for the whole
// kernel, so the scalar data cache may serve it, and the parse then never waits on the vector
// memory counter -- which on gfx9 also counts this wave's output stores (the compiler cannot prove
// the payload unclobbered by those stores, so it would otherwise emit vector loads).  Loads only;
// nothing is ever written through the scalar cache.  Bytes p .. p+4 are valid in the result.
__device__ __forceinline__ uint64_t sload8(const uint32_t* w4, uint32_t p) {
  uint64_t v;
  // (restated uniform: free when the compiler already holds them in SGPRs, and the "s" constraints
  // below cannot take a VGPR where its divergence analysis loses track)
  const uint32_t off = uni(p);
  const uint32_t* const base = reinterpret_cast<const uint32_t*>(uni64(reinterpret_cast<uintptr_t>(w4)));
  asm volatile("s_load_dwordx2 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(base), "s"(off));
  return v >> (8 * (p & 3));
}

// L2 prefetch of the compressed stream ahead of the parse: one wave-wide load, a dword per lane
// 64 bytes apart (4 KiB of stream), issued as an LDS-DMA load (global_load_lds_dword into a 256-byte
// sink nobody reads) so no VGPR waits for it -- the parse's scalar loads then miss the scalar cache
// into L2 instead of into HBM.  The waits it can cause: an LDS access the compiler cannot tell apart
// from the sink waits for the vector memory counter, i.e. the next batch publish (~64 sequences on).
constexpr uint32_t kPfSpan = 4096;   // stream bytes per prefetch
constexpr uint32_t kPfLead = 8192;   // keep the prefetch this far ahead of the parse

__device__ __forceinline__ void prefetch_stream(const uint32_t* w4, uint32_t pos, uint32_t end, uint32_t* sink,
                                                uint32_t lane) {
  const uint32_t q = pos + lane * (kPfSpan / kWave);
  if (q < end)
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(w4 + (q >> 2)),
                                     (__attribute__((address_space(3))) void*)sink, 4, 0, 0);
}

// Parse one LZ4 frame chunk into batches of records, handing each full batch to `flush` (which
// executes it here, or passes it to a consumer wave in k_lz4_pair); returns 0 or an error code.
// The caller checks the decoded size.
template <class Flush>
__device__ __forceinline__ uint32_t parse_frame(Ctx& X, uint32_t lane, Flush&& flush) {
  const uint32_t k0 = uint32_t(reinterpret_cast<uintptr_t>(X.pay) & 3);  // stream pos = k0 + byte index
  const uint32_t* w4 = reinterpret_cast<const uint32_t*>(X.pay - k0);
  const uint32_t end = k0 + X.clen;
  if (X.clen < 7) return ZG_ERR_LZ4;
  if (uint32_t(sload8(w4, k0)) != 0x184D2204u) return ZG_ERR_LZ4;
  const uint32_t flg = uint32_t(sload8(w4, k0 + 4)) & 0xFF;
  if ((flg >> 6) != 1) return ZG_ERR_LZ4;
  uint32_t ip = k0 + 7 + ((flg & 8) ? 8 : 0) + ((flg & 1) ? 4 : 0);
  const uint32_t bck = (flg & 0x10) ? 4 : 0;
  Batch B{0, 0, 0, 0};
  uint32_t pf = ip;  // stream position up to which the prefetch is issued
  while (true) {
    if (B.n > kFlushAbove && !flush(B)) return ZG_ERR_LZ4;
    if (X.pf && pf < end && pf < ip + kPfLead) {
      prefetch_stream(w4, pf, end, X.pf, lane);
      pf += kPfSpan;
    }
    if (ip > end || end - ip < 4) return ZG_ERR_LZ4;
    const uint32_t bs = uint32_t(sload8(w4, ip));
    ip += 4;
    if (bs == 0) break;
    const uint32_t len = bs & 0x7FFFFFFFu;
    if (len > end - ip) return ZG_ERR_LZ4;
    if (bs >> 31) {  // stored block
      emit(B, lane, ip, len, 0, 0);
      ip += len;
    } else {
      const uint32_t bend = uni(ip + len);
      while (true) {
        // loop-carried parse state is wave-uniform; the compiler's uniformity analysis loses track
        // of it through the batch execution inlined into this loop, so restate it (one
        // v_readfirstlane each) and keep every compare and branch of the parse on the scalar unit
        ip = uni(ip);
        B.n = uni(B.n);
        if (B.n > kFlushAbove && !flush(B)) return ZG_ERR_LZ4;
        if (X.pf && pf < end && pf < ip + kPfLead) {  // (after the flush: its LDS waits come a batch later)
          prefetch_stream(w4, pf, end, X.pf, lane);
          pf = uni(pf + kPfSpan);
        }
        if (ip >= bend) return ZG_ERR_LZ4;
        // Fast loop over the common short sequence (literals < 15, match < 19: no length bytes):
        // one 8-byte read at the end of its literals gives the offset and the NEXT token, so the
        // dependent chain is one scalar load per sequence; records go straight into lane n.
        {
          // A fast sequence advances ip by at most 17 bytes, so `iters` of them are known to stay
          // >= 18 bytes before the block end (never the last sequence) and inside the batch:
          // one counter instead of two bounds tests per sequence.
          const uint32_t lim_blk = uni(bend > 18 ? bend - 18 : 0u);
          uint32_t rl = B.rl, rh = B.rh;
          uint32_t token = uint32_t(sload8(w4, ip)) & 0xFF;
          const uint32_t iters0 = uni(ip < lim_blk ? min(kWave - B.n, (lim_blk - ip + 16) / 17) : 0u);
          uint32_t iters = iters0;
          // the record's lane counts down in a VGPR (lane - n): one VALU op per sequence instead of
          // a scalar increment on the CU's one scalar unit, which bounds this loop; the sequences
          // left in the counted run are read off the same countdown (lim_v + dn, equal on every
          // lane), so the loop spends no scalar instruction on its own count either
          int32_t dn = int32_t(lane) - int32_t(B.n);
          const int32_t lim_v = int32_t(iters0) + int32_t(B.n) - int32_t(lane);
          // single-exit loop (a `break` makes the structurizer route the exit flag through VALU)
          // continue while iters > 0 and neither nibble is 15: one integer test (min of the three),
          // computed by the vector unit from a VGPR copy of the loaded bytes (the scalar unit, which
          // bounds this loop, only compares the result)
          uint32_t go = uni(min(min(iters, (token & 15) ^ 15), (token >> 4) ^ 15));
          uint32_t lit = token >> 4;
          uint32_t lp = ip + 1;  // literal position of the current sequence (its token is at lp - 1)
          while (go != 0) {
            const uint32_t p = lp + lit;
            const uint32_t y = uint32_t(sload8(w4, p));  // offset lo, offset hi, next token
            uint32_t yv;
            asm volatile("v_mov_b32 %0, %1" : "=v"(yv) : "s"(y));
            const bool me = dn == 0;
            rl = me ? lp : rl;  // short record: the literals' position (rx stays 0)
            rh = me ? yv : rh;
            lp = p + 3;
            --dn;
            lit = (y >> 20) & 15;  // the next token's literal count: all the scalar unit needs of it
            const uint32_t tv = yv >> 16;
            uint32_t rem;  // counted sequences left (an asm add: the compiler would rebuild a scalar count)
            asm volatile("v_add_u32 %0, %1, %2" : "=v"(rem) : "v"(lim_v), "v"(dn));
            go = __builtin_amdgcn_readfirstlane(min(min(rem, (~tv) & 15), ((tv >> 4) & 15) ^ 15));
          }
          iters = uni(uint32_t(lim_v + dn));
          ip = uni(lp - 1);
          const uint32_t n = uni(B.n + (iters0 - iters));
          B.n = n;
          B.rl = rl;
          B.rh = rh;
          // batch full (execute) or the counted run used up while still clear of the block end
          // (count again): back to the top; a long-length or near-block-end sequence takes the
          // general path (with room for its split records)
          if (n > kFlushAbove || (iters == 0 && ip < lim_blk)) continue;
        }
        const uint32_t token = uint32_t(sload8(w4, ip)) & 0xFF;
        ++ip;
        uint32_t lit = token >> 4, ml = token & 15;
        if (lit == 15) {
          uint32_t b;
          do {
            if (ip >= bend || lit > kMaxChunk) return ZG_ERR_LZ4;
            b = uint32_t(sload8(w4, ip)) & 0xFF;
            ++ip;
            lit += b;
          } while (b == 255);
        }
        if (lit > bend - ip) return ZG_ERR_LZ4;
        const uint32_t lp = ip;
        ip += lit;
        if (ip == bend) {  // last sequence of the block: literals only
          emit(B, lane, lp, lit, 0, 0);
          break;
        }
        if (bend - ip < 2) return ZG_ERR_LZ4;
        const uint32_t off = uint32_t(sload8(w4, ip)) & 0xFFFF;
        ip += 2;
        if (ml == 15) {
          uint32_t b;
          do {
            if (ip >= bend || ml > kMaxChunk) return ZG_ERR_LZ4;
            b = uint32_t(sload8(w4, ip)) & 0xFF;
            ++ip;
            ml += b;
          } while (b == 255);
        }
        emit(B, lane, lp, lit, ml + 4, off);
      }
    }
    ip += bck;
  }
  if (B.n && !flush(B)) return ZG_ERR_LZ4;
  return 0u;
}

// Decode one LZ4 frame chunk with this wave alone; returns 0 or an error code.
__device__ uint32_t decode_chunk(Ctx& X, uint32_t lane) {
  const uint32_t code = parse_frame(X, lane, [&](Batch& B) { return exec_batch(B, X, lane); });
  if (code) return code;
  return X.obase == X.ulen ? 0u : uint32_t(ZG_ERR_SIZE);
}

// amdgpu_waves_per_eu(8): keep 8 waves per SIMD (<= 64 VGPRs).  The decoder is occupancy-bound
// (profiles/lz4_records_r3.md), and with the wide literal copy inlined the register allocator
// otherwise settled on 127 VGPRs = 4 waves per SIMD (hipcc -Rpass-analysis=kernel-resource-usage).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) k_lz4_batched(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                     const ZgChunk* __restrict__ chunks, int n_chunks,
                                                     unsigned long long* err, uint64_t src_n, uint64_t dst_n) {
  __shared__ uint32_t heads[kWavesPerBlock][kWave];
  __shared__ __attribute__((aligned(16))) uint8_t rings[kWavesPerBlock][kRing];
  const uint32_t lane = lane_id();
  const int wave = int(uni(threadIdx.x >> 6));
  const int stride = int(gridDim.x) * kWavesPerBlock;
  for (int c = int(uni(blockIdx.x * kWavesPerBlock + uint32_t(wave))); c < n_chunks; c += stride) {
    ZgChunk ch = chunks[c];
    // the descriptor is wave-uniform: say so, so the whole parse runs on SGPRs / the scalar unit
    // (a vector load would otherwise make every derived position a VGPR and every branch divergent)
    ch.src = uni64(ch.src);
    ch.dst = uni64(ch.dst);
    ch.clen = uni(ch.clen);
    ch.ulen = uni(ch.ulen);
    ch.scheme = uni(ch.scheme);
    if (ch.scheme == 0) continue;
    if (ch.src + ch.clen > src_n || ch.dst + ch.ulen > dst_n) {
      if (lane == 0) report(err, ZG_ERR_RANGE, uint32_t(c));
      continue;
    }
    if (ch.ulen > kMaxChunk) {
      if (lane == 0) report(err, ZG_ERR_CAPACITY, uint32_t(c));
      continue;
    }
    Ctx X;
    X.pay = src + ch.src;
    X.out = dst + ch.dst;
    X.clen = ch.clen;
    X.ulen = ch.ulen;
    X.bg4 = ch.scheme == 2;
    const uint32_t q = ch.ulen >> 2, r = ch.ulen & 3;
    X.g1 = q + (r > 0 ? 1u : 0u);
    X.g2 = X.g1 + q + (r > 1 ? 1u : 0u);
    X.g3 = X.g2 + q + (r > 2 ? 1u : 0u);
    X.k0 = uint32_t(reinterpret_cast<uintptr_t>(X.pay) & 3);
    X.obase = 0;
    X.heads = heads[wave];
    X.ring = rings[wave];
    const uint32_t code = decode_chunk(X, lane);
    if (code && lane == 0) report(err, code, uint32_t(c));
  }
}

// BG4 staging.  Decoding a BG4 chunk straight into its interleaved place writes
// every output line in four passes a quarter-chunk apart (group g's byte p lands at 4 p + g), so each
// 128 B line reached HBM up to four times: 1105 MB of writes for 268 MB of output on 256 MiB of bf16
// (profiles/r5/pmc_table_gpubench256_merkle_stride33_r5i.md).  With a staging slice (one per block,
// kMaxChunk bytes) the consumer decodes the grouped stream there -- contiguous stores, far matches
// read back contiguously, the slice reused chunk after chunk so it stays in L2 / MALL -- and then
// writes the chunk's final bytes once, whole lines at a time: lane i of each step gathers bytes
// 4i .. 4i + 3 of the four groups (one dword each when the group start allows, else bytes) and
// stores the 16 interleaved output bytes.  The fused hash then reads the final bytes from L2.
__device__ __forceinline__ uint32_t load4(const uint8_t* p, bool aligned) {
  if (aligned) return *reinterpret_cast<const uint32_t*>(p);
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

__device__ void ungroup_bg4(const uint8_t* __restrict__ st, uint8_t* __restrict__ out, uint32_t ulen, uint32_t g1,
                            uint32_t g2, uint32_t g3, uint32_t lane) {
  const uint32_t q = ulen >> 2, r = ulen & 3;
  const bool a1 = (g1 & 3) == 0, a2 = (g2 & 3) == 0, a3 = (g3 & 3) == 0;  // group starts (slice is aligned)
  const bool oal = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  const uint32_t q4 = q & ~3u;  // whole 4-index steps
  // four steps' loads are issued before any of their stores: the staged bytes come back from L2, and
  // one step at a time left every step waiting out a full L2 round trip
  constexpr uint32_t kU = 4;
  auto step = [&](uint32_t p0, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t d0 = (a & 0xFFu) | (b & 0xFFu) << 8 | (c & 0xFFu) << 16 | (d & 0xFFu) << 24;
    const uint32_t d1 = (a >> 8 & 0xFFu) | (b & 0xFF00u) | (c & 0xFF00u) << 8 | (d & 0xFF00u) << 16;
    const uint32_t d2 = (a >> 16 & 0xFFu) | (b >> 8 & 0xFF00u) | (c & 0xFF0000u) | (d & 0xFF0000u) << 8;
    const uint32_t d3 = (a >> 24) | (b >> 16 & 0xFF00u) | (c >> 8 & 0xFF0000u) | (d & 0xFF000000u);
    uint8_t* o = out + 4 * p0;
    if (oal) {
      *reinterpret_cast<uint4*>(o) = make_uint4(d0, d1, d2, d3);
    } else {
      const uint32_t w[4] = {d0, d1, d2, d3};
#pragma unroll
      for (int i = 0; i < 16; ++i) o[i] = uint8_t(w[i >> 2] >> (8 * (i & 3)));
    }
  };
  uint32_t p0 = 4 * lane;
  for (; p0 + (kU - 1) * 4 * kWave < q4; p0 += kU * 4 * kWave) {
    uint32_t a[kU], b[kU], c[kU], d[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t p = p0 + u * 4 * kWave;
      a[u] = *reinterpret_cast<const uint32_t*>(st + p);
      b[u] = load4(st + g1 + p, a1);
      c[u] = load4(st + g2 + p, a2);
      d[u] = load4(st + g3 + p, a3);
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) step(p0 + u * 4 * kWave, a[u], b[u], c[u], d[u]);
  }
  for (; p0 < q4; p0 += 4 * kWave)
    step(p0, *reinterpret_cast<const uint32_t*>(st + p0), load4(st + g1 + p0, a1), load4(st + g2 + p0, a2),
         load4(st + g3 + p0, a3));
  // the last q - q4 indices of every group, then the r leftover bytes (groups 0 .. r-1 hold one more)
  const uint32_t tail = 4 * (q - q4) + r;
  if (lane < tail) {
    const uint32_t pos = 4 * q4 + lane;  // output position
    const uint32_t g = pos & 3, p = pos >> 2;
    const uint32_t gs = g == 0 ? 0u : g == 1 ? g1 : g == 2 ? g2 : g3;
    out[pos] = st[gs + p];
  }
}

// -----------------------------------------------------------------------------------------------
// Producer/consumer pairs (k_lz4_pair): two waves per chunk.  The one-wave decoder alternates its
// scalar parse of 64 sequences with their lane-parallel execution, so a chunk's latency is the SUM of
// the two halves; a launch with fewer chunks than resident waves (a 256 MiB batch is ~4 k chunks
// against 8 k wave slots, the tail rounds of a pull fewer still) leaves that latency exposed.  Here
// wave 0 of a block parses (parse_frame, unchanged) and publishes each full batch into an LDS ring
// of kPairSlots slots; wave 1 takes the batches in order and runs exec_batch (its own heads / history
// ring / output position), so parse and execute of a chunk overlap on two SIMDs and the chip holds
// twice the waves for the same chunk count.  Slot hand-off: a batch number q uses slot q % R; the
// producer waits until the slot was consumed q / R times, writes the records, then (release) marks
// it full; the consumer waits for full (acquire), copies the records out, marks it consumed.  Every
// chunk ends with an end marker carrying the parse status; a consumer whose exec_batch fails sets
// the chunk's abort mark (the producer stops at its next publish) and drains to the end marker.
// Every wait is bounded (kPairSpinMax sleeps): a protocol bug cannot hang the GPU -- the block
// reports ZG_ERR_LZ4 and leaves.
constexpr uint32_t kPairSlots = 4;
constexpr uint32_t kPairEnd = 0x80000000u;   // n field of an end marker (| status code)
constexpr uint32_t kPairSpinMax = 1u << 22;  // ~0.1 s of s_sleep 1
// Ticket ring of the dynamic chunk schedule.  Every ticketed chunk publishes at least its end marker,
// and the producer is at most kPairSlots publishes ahead of the consumer, so it is never more than
// kPairSlots + 1 tickets ahead: 8 entries are never overwritten unread.
constexpr uint32_t kPairTickets = 8;

struct PairLds {
  uint32_t rl[kPairSlots][kWave], rh[kPairSlots][kWave], rx[kPairSlots][kWave];
  uint32_t n[kPairSlots];
  uint32_t full[kPairSlots];  // times the producer filled the slot
  uint32_t done[kPairSlots];  // times the consumer emptied it
  uint32_t abort;             // chunk index + 1 whose execution failed
  uint32_t dead;              // a wait ran out: both waves leave
  uint32_t heads[kWave];
  uint32_t ticket[kPairTickets];  // dynamic scheduling: the chunk of the block's k-th ticket
  uint32_t tseq[kPairTickets];    // k + 1 once ticket k is written
  uint32_t pf[kWave];             // the producer's stream-prefetch sink (written, never read)
  __attribute__((aligned(16))) uint8_t ring[kRing];
};

__device__ __forceinline__ uint32_t lds_acquire(const uint32_t* p) {
  return uni(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}

__device__ __forceinline__ void lds_release(uint32_t* p, uint32_t v, uint32_t lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Wait until *p == want; false (and the block marked dead) when the wait runs out.
__device__ __forceinline__ bool lds_wait(PairLds& L, const uint32_t* p, uint32_t want, uint32_t lane) {
  for (uint32_t k = 0; lds_acquire(p) != want; ++k) {
    if (k > kPairSpinMax || lds_acquire(&L.dead)) {
      lds_release(&L.dead, 1u, lane);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// (8 waves per SIMD: see k_lz4_batched)
//
// hashes != nullptr: the consumer also computes each chunk's Xet BLAKE3 hash (hashes[c], 32 bytes;
// sizes[c] = its length) as soon as the chunk is decoded -- one wave over the output it just wrote,
// which is still in L2, with the history ring as the chaining-value scratch -- so the chunk never
// needs a hash pass of its own (the fused place/hash pass then covers stored chunks only).  The
// decoder issues little VALU work (~15 % of wave-cycles), so the hashing mostly fills idle issue
// slots; only the last chunks' hashes add to the launch.  A chunk that fails hashes as all-ones.
// (A template: kHash = false is the decode-only kernel, register allocation untouched by the hash.)
// (kDiag: the diagnostics build -- `dbg` bits read; the production kernels compile them out, so the
// flags cost them no registers)
// Kernel arguments of k_lz4_pair.  The kernel reads each field from the kernarg segment where it
// uses it (pair_args(): an opaque copy of the segment pointer per use, so no field is hoisted and
// held in a register across the decode loops) -- the producer's parse keeps ~80 SGPRs busy, and
// arguments held live across it were spilled to VGPR lanes and from there to scratch memory.
struct PairArgs {
  const uint8_t* src;
  uint8_t* dst;
  const ZgChunk* chunks;
  unsigned long long* err;
  uint64_t src_n, dst_n;
  uint8_t* hashes;
  uint64_t* sizes;
  uint8_t* stage;
  uint32_t* work;
  int n_chunks;
  uint32_t dbg;
  uint32_t prefetch;  // the producer's stream prefetch (ZG_PAIR_PREFETCH=0: off, for A/Bs)
};
typedef const __attribute__((address_space(4))) PairArgs* PairArgsPtr;

__device__ __forceinline__ PairArgsPtr pair_args() {
  PairArgsPtr p = (PairArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

template <bool kHash, bool kDiag>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(8, 8))) k_lz4_pair(const PairArgs args) {
  __shared__ PairLds L;
  const uint32_t lane = lane_id();
  const bool producer = uni(threadIdx.x >> 6) == 0;
  if (threadIdx.x < kPairSlots) L.full[threadIdx.x] = L.done[threadIdx.x] = 0;
  if (threadIdx.x < kPairTickets) L.tseq[threadIdx.x] = 0;
  if (threadIdx.x == 0) L.abort = L.dead = 0;
  __syncthreads();
  uint32_t q = 0;  // batch sequence number, counted identically by both waves
  // Chunk schedule.  Static (work == nullptr): block b takes chunks b, b + grid, ...  Dynamic: the
  // producer takes the next chunk from the launch's work counter (one vector atomic from lane 0)
  // whenever it starts one, and hands it to the consumer through the LDS ticket ring -- a block that
  // finished a small chunk takes the next one at once, so a launch is no longer as long as the
  // blocks that were dealt one chunk more than the others (a 256 MiB batch: ~4.2 k chunks on 4096
  // blocks, 98 of them decoding two in a row, tools/gpu/lz4_split_probe.py).  Stored chunks and
  // chunks that fail the range checks never get a ticket: the producer settles them itself.
  uint32_t tk = 0;  // chunks taken: dynamic, tickets; static, block b's k-th chunk is b + k * grid
  while (true) {
    const PairArgsPtr A = pair_args();
    const int n_chunks = A->n_chunks;
    int c;
    if (A->work != nullptr) {
      const uint32_t slot = tk % kPairTickets;
      if (producer) {
        while (true) {
          uint32_t v = 0;
          if (lane == 0) v = atomicAdd(A->work, 1u);
          c = int(uni(v));
          if (c >= n_chunks) break;
          const ZgChunk h = A->chunks[c];
          const uint32_t sc = uni(h.scheme), cl = uni(h.clen), ul = uni(h.ulen);
          const uint64_t so = uni64(h.src), dso = uni64(h.dst);
          if (sc == 0) continue;
          const bool range_bad = so + cl > A->src_n || dso + ul > A->dst_n;
          if (range_bad || ul > kMaxChunk) {
            if (lane == 0) report(pair_args()->err, range_bad ? ZG_ERR_RANGE : ZG_ERR_CAPACITY, uint32_t(c));
            if (kHash) {
              if (lane < 8) reinterpret_cast<uint32_t*>(pair_args()->hashes + 32 * uint64_t(c))[lane] = 0xFFFFFFFFu;
              if (pair_args()->sizes && lane == 0) pair_args()->sizes[c] = 0;
            }
            continue;
          }
          break;
        }
        if (lane == 0) L.ticket[slot] = uint32_t(c < n_chunks ? c : n_chunks);
        lds_release(&L.tseq[slot], tk + 1u, lane);
      } else {
        if (!lds_wait(L, &L.tseq[slot], tk + 1u, lane)) return;
        c = int(uni(L.ticket[slot]));
      }
      ++tk;
    } else {
      c = int(uni(blockIdx.x + tk * gridDim.x));
      ++tk;
    }
    if (c >= n_chunks) break;
    ZgChunk ch = A->chunks[c];
    ch.src = uni64(ch.src);
    ch.dst = uni64(ch.dst);
    ch.clen = uni(ch.clen);
    ch.ulen = uni(ch.ulen);
    ch.scheme = uni(ch.scheme);
    if (ch.scheme == 0) continue;
    auto bad_hash = [&]() {  // (consumer) a chunk that is not decoded hashes as all-ones
      if (!kHash) return;
      if (lane < 8) reinterpret_cast<uint32_t*>(pair_args()->hashes + 32 * uint64_t(c))[lane] = 0xFFFFFFFFu;
      if (pair_args()->sizes && lane == 0) pair_args()->sizes[c] = 0;
    };
    if (ch.src + ch.clen > A->src_n || ch.dst + ch.ulen > A->dst_n) {
      if (!producer && lane == 0) report(pair_args()->err, ZG_ERR_RANGE, uint32_t(c));
      if (!producer) bad_hash();
      continue;
    }
    if (ch.ulen > kMaxChunk) {
      if (!producer && lane == 0) report(pair_args()->err, ZG_ERR_CAPACITY, uint32_t(c));
      if (!producer) bad_hash();
      continue;
    }
    Ctx X;
    X.pay = A->src + ch.src;
    X.out = A->dst + ch.dst;
    X.clen = ch.clen;
    X.ulen = ch.ulen;
    X.bg4 = ch.scheme == 2;
    const uint32_t qq = ch.ulen >> 2, r = ch.ulen & 3;
    X.g1 = qq + (r > 0 ? 1u : 0u);
    X.g2 = X.g1 + qq + (r > 1 ? 1u : 0u);
    X.g3 = X.g2 + qq + (r > 2 ? 1u : 0u);
    X.k0 = uint32_t(reinterpret_cast<uintptr_t>(X.pay) & 3);
    X.obase = 0;
    X.heads = L.heads;
    X.ring = L.ring;
    // BG4 with a staging slice: decode the grouped stream contiguously into it (see ungroup_bg4)
    const bool staged = A->stage != nullptr && X.bg4;
    if (staged) {
      X.out = A->stage + size_t(blockIdx.x) * kMaxChunk;
      X.bg4 = false;
    }
    const uint32_t cmark = uint32_t(c) + 1u;
    if (producer) {
      X.pf = pair_args()->prefetch ? L.pf : nullptr;
      bool alive = true;
      auto publish = [&](uint32_t n, uint32_t rl, uint32_t rh, uint32_t rx) -> bool {
        q = uni(q);  // (wave-uniform: keeps the slot waits on the scalar unit)
        const uint32_t slot = q & (kPairSlots - 1), uses = q / kPairSlots;
        if (!lds_wait(L, &L.done[slot], uses, lane)) return alive = false;
        L.rl[slot][lane] = rl;
        L.rh[slot][lane] = rh;
        L.rx[slot][lane] = rx;
        if (lane == 0) L.n[slot] = n;
        lds_release(&L.full[slot], uses + 1u, lane);
        ++q;
        return true;
      };
      const uint32_t code = parse_frame(X, lane, [&](Batch& B) {
        if (lds_acquire(&L.abort) == cmark) return false;  // the consumer failed this chunk: stop
        const bool ok = publish(B.n, B.rl, B.rh, B.rx);
        B.n = 0;
        B.rl = B.rh = B.rx = 0;
        return ok;
      });
      // the prefetches' LDS writes land before the block can exit (and its LDS be reallocated)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!alive || !publish(kPairEnd | code, 0u, 0u, 0u)) return;
    } else {
      bool failed = false, whole = false;
      while (true) {
        q = uni(q);  // (wave-uniform: keeps the slot waits on the scalar unit)
        const uint32_t slot = q & (kPairSlots - 1), uses = q / kPairSlots;
        if (!lds_wait(L, &L.full[slot], uses + 1u, lane)) {
          if (lane == 0) report(pair_args()->err, ZG_ERR_LZ4, uint32_t(c));
          bad_hash();
          return;
        }
        Batch B;
        B.n = uni(L.n[slot]);
        B.rl = L.rl[slot][lane];
        B.rh = L.rh[slot][lane];
        B.rx = L.rx[slot][lane];
        lds_release(&L.done[slot], uses + 1u, lane);
        ++q;
        if (B.n & kPairEnd) {
          const uint32_t code = B.n & ~kPairEnd;
          if (!failed) {
            if (code) {
              if (lane == 0) report(pair_args()->err, code, uint32_t(c));
            } else if (X.obase != X.ulen) {
              if (lane == 0) report(pair_args()->err, ZG_ERR_SIZE, uint32_t(c));
            } else {
              whole = true;
            }
          }
          break;
        }
        // (dbg & 1, diagnostics only: the consumer takes the records without executing them -- the
        // launch then times the parse alone, tools/gpu/lz4_split_probe.py; the chunk reports a size error)
        if (!failed && !(kDiag && (pair_args()->dbg & 1u)) && !exec_batch(B, X, lane)) {
          failed = true;
          if (lane == 0) report(pair_args()->err, ZG_ERR_LZ4, uint32_t(c));
          lds_release(&L.abort, cmark, lane);
        }
      }
      if (kDiag && (pair_args()->dbg & 2u)) whole = false;  // (diagnostics: execute only -- no ungroup, no hash)
      if (staged) {
        // (the chunk's final place re-read, not held across the batch loop)
        uint8_t* const final_out = pair_args()->dst + uni64(pair_args()->chunks[c].dst);
        if (whole) {
          // the staged stream is complete in L2 (this wave's stores acknowledged, L1 dropped): write
          // the chunk's final bytes once
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          ungroup_bg4(X.out, final_out, X.ulen, X.g1, X.g2, X.g3, lane);
        }
        X.out = final_out;
        // the next chunk of this block decodes into the same slice: every lane's reads of it done
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
      }
      if (kHash) {
        if (whole) {
          // this wave wrote every output byte: its stores acknowledged (vmcnt also counts stores),
          // then L1 invalidated, so the hash reads them back from L2
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          uint32_t h[8];
          zg::wave_hash(X.out, X.ulen, zg::kDataKeyW, zg::KEYED_HASH, reinterpret_cast<uint32_t*>(L.ring), lane, h);
          zg::store_hash(pair_args()->hashes + 32 * uint64_t(c), h, lane);
          if (pair_args()->sizes && lane == 0) pair_args()->sizes[c] = X.ulen;
          __builtin_amdgcn_wave_barrier();  // the next chunk's exec_batch reuses the ring
        } else {
          bad_hash();
        }
      }
    }
  }
}

// -----------------------------------------------------------------------------------------------
// Experimental two-kernel decode: SIMT parse (a LANE per chunk) + record-driven execute (a WAVE per
// chunk).  Not on the ingest path: reachable through zg_lz4_decode_records / hip().lz4_decode(...,
// rec_scratch=...) for kbench and tests.
//
// Why it exists: the wave-per-chunk decoder above parses on the scalar unit (~22 SALU per
// sequence; a CU has one scalar unit for its 4 SIMDs), and on BG4 bf16 (~6.8k sequences per
// 64 KiB) 1 GiB took 11.1 ms at 8 waves/SIMD, 14.7 at 4, 21.4 at 2.  Here the parse is vector code
// with one lane per chunk, every sequence becomes an 8-byte record {literal position | literal
// length << 18, offset | match length << 16} in a scratch region owned by the chunk (3/8 record
// per compressed byte: LZ4 needs >= 3 bytes per sequence), and the execute kernel loads 64 records
// per batch with one vector load and runs exec_batch.  A chunk whose parse fails or does not fit
// its region gets count kNoRecs and is decoded by decode_chunk, which reports the exact error.
//
// Measured on MI355X (profiles/lz4_records_r3.md, 1 GiB of BG4 bf16): the execute kernel alone
// takes 6.4 ms (1.75x faster than the one-kernel decoder's 11.1), but the parse takes 15 ms: only
// 16.7k chunks = 261 waves of lanes, each walking ~6.8k sequences through dependent loads, and the
// compiler's vmcnt(0) waits inside the divergent loop also wait for the record stores.  A parse
// that stages each lane's stream in LDS in bulk would be the next step.
constexpr uint32_t kNoRecs = 0xFFFFFFFFu;
constexpr uint32_t kRecLitMax = 0x3FFFu;  // 14-bit literal field
constexpr uint32_t kRecMlMax = 0x7FFFu;

__host__ __device__ inline uint64_t rec_index(uint64_t src_off) { return (3 * src_off) >> 3; }

// Per-lane reader over a payload [base, base + clen): 4 bytes at index p as two aligned dword loads
// (the streams are sequential per lane, so these hit the vector L1 after the first touch) joined
// by v_alignbyte.  The high dword's address is clamped to the payload's last dword, so nothing
// past the buffer is touched (its bytes past the payload never decide anything).  Plain values
// only: a register window selected by lane-varying indices was lowered to scratch memory.
struct LaneRd {
  const uint8_t* w;  // payload rounded down to a dword
  uint32_t k0;       // payload address & 3
  uint32_t last;     // index (from w) of the payload's last dword
};

__device__ __forceinline__ uint32_t rd4(const LaneRd& r, uint32_t p) {
  const uint32_t q = (r.k0 + p) & ~3u;
  const uint32_t lo = *reinterpret_cast<const uint32_t*>(r.w + q);
  const uint32_t hi = *reinterpret_cast<const uint32_t*>(r.w + min(q + 4, r.last));
  return __builtin_amdgcn_alignbyte(hi, lo, (r.k0 + p) & 3);  // byte shift
}

struct RecOut {
  uint2* rec;
  uint32_t n, cap;
  bool over;
};

__device__ __forceinline__ void rec_emit(RecOut& o, uint32_t lp, uint32_t lit, uint32_t ml, uint32_t off) {
  do {
    const uint32_t l = lit > kRecLitMax ? kRecLitMax : lit;
    const uint32_t m = lit > kRecLitMax ? 0u : (ml > kRecMlMax ? kRecMlMax : ml);
    if (o.n < o.cap) o.rec[o.n] = make_uint2(lp | (l << 18), off | (m << 16));
    else o.over = true;
    ++o.n;
    lp += l;
    lit -= l;
    ml -= m;
  } while (lit | ml);
}

// Parse one chunk's LZ4 frame into records; returns the record count or kNoRecs.
__device__ uint32_t parse_chunk(const uint8_t* pay, uint32_t clen, uint2* rec, uint32_t cap) {
  LaneRd r;
  r.k0 = uint32_t(reinterpret_cast<uintptr_t>(pay) & 3);
  r.w = pay - r.k0;
  r.last = (r.k0 + (clen ? clen - 1 : 0)) & ~3u;
  RecOut o{rec, 0u, cap, false};
  if (clen < 7 || rd4(r, 0) != 0x184D2204u) return kNoRecs;
  const uint32_t flg = rd4(r, 4) & 0xFF;
  if ((flg >> 6) != 1) return kNoRecs;
  uint32_t ip = 7 + ((flg & 8) ? 8 : 0) + ((flg & 1) ? 4 : 0);
  const uint32_t bck = (flg & 0x10) ? 4 : 0;
  while (true) {
    if (ip > clen || clen - ip < 4) return kNoRecs;
    const uint32_t bs = rd4(r, ip);
    ip += 4;
    if (bs == 0) break;
    const uint32_t len = bs & 0x7FFFFFFFu;
    if (len > clen - ip) return kNoRecs;
    if (bs >> 31) {  // stored block: literals only
      if (len) rec_emit(o, ip, len, 0, 0);
      ip += len;
    } else {
      const uint32_t bend = ip + len;
      while (true) {
        if (ip >= bend) return kNoRecs;
        const uint32_t t = rd4(r, ip);  // token + the 3 bytes after it
        const uint32_t token = t & 0xFF;
        ++ip;
        uint32_t lit = token >> 4, ml = token & 15;
        if (lit == 15) {
          uint32_t b;
          do {
            if (ip >= bend || lit > kMaxChunk) return kNoRecs;
            b = rd4(r, ip) & 0xFF;
            ++ip;
            lit += b;
          } while (b == 255);
        }
        if (lit > bend - ip) return kNoRecs;
        const uint32_t lp = ip;
        ip += lit;
        if (ip == bend) {  // last sequence of the block: literals only
          if (lit) rec_emit(o, lp, lit, 0, 0);
          break;
        }
        if (bend - ip < 2) return kNoRecs;
        const uint32_t off = (lit == 0 ? t >> 8 : rd4(r, ip)) & 0xFFFF;  // no literals: already in t
        ip += 2;
        if (ml == 15) {
          uint32_t b;
          do {
            if (ip >= bend || ml > kMaxChunk) return kNoRecs;
            b = rd4(r, ip) & 0xFF;
            ++ip;
            ml += b;
          } while (b == 255);
        }
        rec_emit(o, lp, lit, ml + 4, off);
      }
    }
    ip += bck;
  }
  return o.over ? kNoRecs : o.n;
}

__global__ void __launch_bounds__(256) k_lz4_parse(const uint8_t* __restrict__ src, const ZgChunk* __restrict__ chunks,
                                                   int n_chunks, uint64_t src_n, uint64_t dst_n, uint2* __restrict__ recs,
                                                   uint32_t* __restrict__ counts) {
  const int c = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (c >= n_chunks) return;
  const ZgChunk ch = chunks[c];
  uint32_t cnt = kNoRecs;
  if (ch.scheme != 0 && ch.src + ch.clen <= src_n && ch.dst + ch.ulen <= dst_n && ch.ulen <= kMaxChunk) {
    const uint64_t r0 = rec_index(ch.src), r1 = rec_index(ch.src + ch.clen);
    cnt = parse_chunk(src + ch.src, ch.clen, recs + r0, uint32_t(r1 - r0));
  }
  counts[c] = cnt;
}

// Execute one chunk's records (64 per batch, the next batch's records loaded while this one runs).
__device__ uint32_t exec_records(Ctx& X, const uint2* rec, uint32_t cnt, uint32_t lane) {
  uint2 nx = lane < cnt ? rec[lane] : make_uint2(0u, 0u);
  for (uint32_t b0 = 0; b0 < cnt; b0 += kWave) {
    const uint2 r = nx;
    const uint32_t i = b0 + kWave + lane;
    nx = i < cnt ? rec[i] : make_uint2(0u, 0u);
    Batch B;
    B.n = uni(min(uint32_t(kWave), cnt - b0));
    B.rl = X.k0 + (r.x & 0x3FFFFu);
    B.rh = r.y & 0xFFFFu;
    B.rx = 0x80000000u | ((r.y >> 16) << 16) | (r.x >> 18);
    if (!exec_batch(B, X, lane)) return ZG_ERR_LZ4;
  }
  return X.obase == X.ulen ? 0u : uint32_t(ZG_ERR_SIZE);
}

__global__ void __launch_bounds__(256) k_lz4_exec(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  const ZgChunk* __restrict__ chunks, int n_chunks,
                                                  unsigned long long* err, uint64_t src_n, uint64_t dst_n,
                                                  const uint2* __restrict__ recs, const uint32_t* __restrict__ counts) {
  __shared__ uint32_t heads[kWavesPerBlock][kWave];
  __shared__ __attribute__((aligned(16))) uint8_t rings[kWavesPerBlock][kRing];
  const uint32_t lane = lane_id();
  const int wave = int(uni(threadIdx.x >> 6));
  const int stride = int(gridDim.x) * kWavesPerBlock;
  for (int c = int(uni(blockIdx.x * kWavesPerBlock + uint32_t(wave))); c < n_chunks; c += stride) {
    ZgChunk ch = chunks[c];
    ch.src = uni64(ch.src);
    ch.dst = uni64(ch.dst);
    ch.clen = uni(ch.clen);
    ch.ulen = uni(ch.ulen);
    ch.scheme = uni(ch.scheme);
    if (ch.scheme == 0) continue;
    if (ch.src + ch.clen > src_n || ch.dst + ch.ulen > dst_n) {
      if (lane == 0) report(err, ZG_ERR_RANGE, uint32_t(c));
      continue;
    }
    if (ch.ulen > kMaxChunk) {
      if (lane == 0) report(err, ZG_ERR_CAPACITY, uint32_t(c));
      continue;
    }
    Ctx X;
    X.pay = src + ch.src;
    X.out = dst + ch.dst;
    X.clen = ch.clen;
    X.ulen = ch.ulen;
    X.bg4 = ch.scheme == 2;
    const uint32_t q = ch.ulen >> 2, r = ch.ulen & 3;
    X.g1 = q + (r > 0 ? 1u : 0u);
    X.g2 = X.g1 + q + (r > 1 ? 1u : 0u);
    X.g3 = X.g2 + q + (r > 2 ? 1u : 0u);
    X.k0 = uint32_t(reinterpret_cast<uintptr_t>(X.pay) & 3);
    X.obase = 0;
    X.heads = heads[wave];
    X.ring = rings[wave];
    const uint32_t cnt = uni(counts[c]);
    const uint32_t code = cnt == kNoRecs ? decode_chunk(X, lane) : exec_records(X, recs + rec_index(ch.src), cnt, lane);
    if (code && lane == 0) report(err, code, uint32_t(c));
  }
}

}  // namespace

extern "C" hipError_t zg_lz4_batched_decode_grid(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                                 const ZgChunk* chunks, int n_chunks, unsigned long long* err,
                                                 int grid_cap, hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  if (grid_cap <= 0 || grid_cap >= 8192) grid_cap = 2048;
  const int blocks = (n_chunks + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_lz4_batched, dim3(blocks < grid_cap ? blocks : grid_cap), dim3(256), 0, stream, src, dst,
                     chunks, n_chunks, err, src_n, dst_n);
  return hipGetLastError();
}

constexpr int kPairGrid = 4096;  // 4096 pairs = 8 waves / SIMD

constexpr size_t kWorkBytes = 256;  // the dynamic schedule's counter (one dword, padded)

// Staging bytes for BG4 chunks of a pair launch over n chunks (one kMaxChunk slice per block), plus
// the dynamic schedule's work counter.
extern "C" size_t zg_lz4_stage_bytes(int n_chunks) {
  if (n_chunks <= 0) return 0;
  return size_t(n_chunks < kPairGrid ? n_chunks : kPairGrid) * kMaxChunk + kWorkBytes;
}

static bool dynamic_enabled() {
  const char* v = getenv("ZG_PAIR_DYNAMIC");  // read per launch: A/B of the chunk schedule
  return !(v && atoi(v) == 0);
}

static uint32_t pair_debug() {
  const char* v = getenv("ZG_PAIR_DEBUG");  // diagnostics (k_lz4_pair `dbg`); unset in every real run
  return v ? uint32_t(atoi(v)) : 0u;
}

static bool stage_enabled() {
  const char* v = getenv("ZG_BG4_STAGE");  // read per launch: tests A/B both paths in one process
  return !(v && atoi(v) == 0);
}

extern "C" hipError_t zg_lz4_pair_decode_hash_staged(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                                     const ZgChunk* chunks, int n_chunks, unsigned long long* err,
                                                     int grid_cap, uint8_t* hashes, uint64_t* sizes, uint8_t* stage,
                                                     size_t stage_bytes, hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  if (grid_cap <= 0 || grid_cap > 8192) grid_cap = kPairGrid;
  const int grid = n_chunks < grid_cap ? n_chunks : grid_cap;
  // the dynamic schedule's work counter lives in the scratch right after the staging slices (the
  // scratch is this pipeline's: its launches are ordered on one stream), zeroed before the launch
  uint32_t* work = nullptr;
  if (stage && dynamic_enabled() && stage_bytes >= size_t(grid) * kMaxChunk + kWorkBytes) {
    work = reinterpret_cast<uint32_t*>(stage + size_t(grid) * kMaxChunk);
    const hipError_t e = hipMemsetAsync(work, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
  }
  if (!stage_enabled() || !stage || stage_bytes < size_t(grid) * kMaxChunk) stage = nullptr;
  const uint32_t dbg = pair_debug();
  const char* pfv = getenv("ZG_PAIR_PREFETCH");  // read per launch: A/B of the stream prefetch
  const uint32_t prefetch = (pfv && atoi(pfv) == 0) ? 0u : 1u;
  const PairArgs args{src, dst, chunks, err, src_n, dst_n, hashes, sizes, stage, work, n_chunks, dbg, prefetch};
  if (hashes && dbg)
    hipLaunchKernelGGL((k_lz4_pair<true, true>), dim3(grid), dim3(2 * kWave), 0, stream, args);
  else if (hashes)
    hipLaunchKernelGGL((k_lz4_pair<true, false>), dim3(grid), dim3(2 * kWave), 0, stream, args);
  else
    hipLaunchKernelGGL((k_lz4_pair<false, false>), dim3(grid), dim3(2 * kWave), 0, stream, args);
  return hipGetLastError();
}

extern "C" hipError_t zg_lz4_pair_decode_hash(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                              const ZgChunk* chunks, int n_chunks, unsigned long long* err, int grid_cap,
                                              uint8_t* hashes, uint64_t* sizes, hipStream_t stream) {
  return zg_lz4_pair_decode_hash_staged(src, src_n, dst, dst_n, chunks, n_chunks, err, grid_cap, hashes, sizes,
                                        nullptr, 0, stream);
}

extern "C" hipError_t zg_lz4_pair_decode(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                         const ZgChunk* chunks, int n_chunks, unsigned long long* err, int grid_cap,
                                         hipStream_t stream) {
  return zg_lz4_pair_decode_hash(src, src_n, dst, dst_n, chunks, n_chunks, err, grid_cap, nullptr, nullptr, stream);
}

extern "C" hipError_t zg_lz4_batched_decode(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                            const ZgChunk* chunks, int n_chunks, unsigned long long* err,
                                            hipStream_t stream) {
  // ZG_LZ4_GRID caps the persistent grid (occupancy experiments); default 2048 blocks = 8 waves/SIMD.
  static const int grid_cap = [] {
    const char* v = getenv("ZG_LZ4_GRID");
    return v ? atoi(v) : 0;
  }();
  // ZG_LZ4_PAIR: 1 (default) = producer/consumer pairs, 0 = the one-wave decoder, auto = pairs for
  // launches of fewer than kPairBelow chunks.  With the wide literal copies and both kernels held at
  // 8 waves per SIMD, pairs win at every size (BG4 bf16, kbench k3pair, one-wave -> pair: 128 MiB
  // 48 -> 78 GB/s, 256 MiB 82 -> 95, 512 MiB 95 -> 124, 1 GiB 123 -> 136;
  // profiles/r4/kbench_k3_wide_r4j.jsonl).  Before them the one-wave decoder won from ~10 k chunks
  // up (profiles/r4/kbench_k3pair_sizes_r4e.jsonl), which is what `auto` keeps.
  constexpr int kPairBelow = 10240;
  static const int pair = [] {
    const char* v = getenv("ZG_LZ4_PAIR");
    if (!v) return 1;
    if (std::string(v) == "auto") return 2;
    return atoi(v) ? 1 : 0;
  }();
  if (pair == 1 || (pair == 2 && n_chunks < kPairBelow))
    return zg_lz4_pair_decode(src, src_n, dst, dst_n, chunks, n_chunks, err, 0, stream);
  return zg_lz4_batched_decode_grid(src, src_n, dst, dst_n, chunks, n_chunks, err, grid_cap, stream);
}

// Decode for an unclipped ingest launch.  With the pair decoder (the default) and ZG_FUSED_HASH not 0,
// every compressed chunk is also hashed by the decoder (hashes[c], sizes[c]) and *hashed is set to
// 1, so the following place/hash pass skips compressed chunks; else *hashed = 0.
extern "C" hipError_t zg_lz4_decode_ingest(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                           const ZgChunk* chunks, int n_chunks, unsigned long long* err,
                                           uint8_t* hashes, uint64_t* sizes, int* hashed, uint8_t* stage,
                                           size_t stage_bytes, hipStream_t stream) {
  const char* v = getenv("ZG_FUSED_HASH");  // read per launch: tests A/B both paths in one process
  const char* p = getenv("ZG_LZ4_PAIR");
  const bool fuse = !(v && atoi(v) == 0) && !(p && std::string(p) != "1");
  *hashed = 0;
  if (!fuse || !hashes) return zg_lz4_batched_decode(src, src_n, dst, dst_n, chunks, n_chunks, err, stream);
  *hashed = 1;
  return zg_lz4_pair_decode_hash_staged(src, src_n, dst, dst_n, chunks, n_chunks, err, 0, hashes, sizes, stage,
                                        stage_bytes, stream);
}

extern "C" size_t zg_lz4_rec_scratch_bytes(int n_chunks, uint64_t src_n) {
  if (n_chunks <= 0) return 0;
  const uint64_t counts = (4 * uint64_t(n_chunks) + 255) & ~uint64_t(255);
  return size_t(counts + 8 * (rec_index(src_n) + 2));
}

extern "C" hipError_t zg_lz4_decode_records(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                            const ZgChunk* chunks, int n_chunks, unsigned long long* err,
                                            uint8_t* scratch, size_t scratch_bytes, hipStream_t stream) {
  if (n_chunks <= 0) return hipSuccess;
  if (!scratch || scratch_bytes < zg_lz4_rec_scratch_bytes(n_chunks, src_n))
    return zg_lz4_batched_decode(src, src_n, dst, dst_n, chunks, n_chunks, err, stream);
  uint32_t* counts = reinterpret_cast<uint32_t*>(scratch);
  uint2* recs = reinterpret_cast<uint2*>(scratch + ((4 * uint64_t(n_chunks) + 255) & ~uint64_t(255)));
  hipLaunchKernelGGL(k_lz4_parse, dim3((n_chunks + 255) / 256), dim3(256), 0, stream, src, chunks, n_chunks, src_n,
                     dst_n, recs, counts);
  const int blocks = (n_chunks + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_lz4_exec, dim3(blocks < 2048 ? blocks : 2048), dim3(256), 0, stream, src, dst, chunks, n_chunks,
                     err, src_n, dst_n, recs, counts);
  return hipGetLastError();
}

