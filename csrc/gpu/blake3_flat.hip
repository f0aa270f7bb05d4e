// K1, leaf-flat: keyed BLAKE3 of many Xet chunks with every lane busy.
//
// Xet chunks are 8-128 KiB (CDC), i.e. 8-128 BLAKE3 chunks ("leaves") of 1 KiB.  The wave-per-Xet-
// chunk kernel (ingest.hip, k_hash_chunks) gives lane l leaf l: a 40-leaf chunk leaves 24 lanes idle
// for all 16 block compressions, a 72-leaf chunk needs a second 16-block pass for 8 lanes, and the
// 6-7 parent levels after that run with 32/16/.../1 lanes.  On the CDC chunks of a real pull that
// kernel ran at 1.4 TB/s (profiles/bench70b_n1_kernels_r2.md), about 40 % of the VALU peak for
// BLAKE3.  Here the work is re-cut so the lanes stay full:
//
//   k_plan_tiles + k_plan_scan
//                  exclusive scan of leaves per chunk -> P[c] (per-tile sums, then per-tile scans
//                  over the whole chip); WF[t] = the chunk that owns leaf 64 t (where wave task t
//                  starts); L = total leaves.
//   k_hash_leaves  lane per leaf over the launch's leaves packed back to back (wave task t = leaves
//                  64t..64t+63, persistent grid, so only the launch's last task has idle lanes);
//                  next block's loads in flight during each compression; chaining values -> CV[g].
//                  A one-leaf chunk is its own root and its hash is written here.
//   k_hash_tree    8 Xet chunks per wave: each level's parent compressions of all 8 chunks are one
//                  flat task list (pairwise with carry == BLAKE3's left-complete tree), in place in
//                  CV; the compression with two nodes left carries ROOT and writes the hash.
//
// Scratch (caller-owned, one per concurrently running launch): 64 B header | P[n+1] | WF[cap/64+2]
// | TS[tiles] | CV[cap][8 words], cap >= total leaves (total_bytes / 1024 + n bounds it).  If the launch has
// more leaves than cap (caller undersized the scratch) every hash is written as 32 x 0xFF, so the
// result cannot verify.
#include <hip/hip_runtime.h>

#include "blake3_dev.h"
#include "wave64.h"
#include "zgpu.h"

namespace {

constexpr int kWave = 64;
constexpr uint32_t kMaxChunk = 128u * 1024u;
constexpr int kTreeG = 8;           // Xet chunks per wave in k_hash_tree
constexpr int kPlanThreads = 1024;  // chunks per plan tile (one per thread)
constexpr int kLeafMaxWaves = 8192; // persistent leaf grid cap (32 waves per CU)

struct PlanHdr {
  uint32_t leaves;    // L
  uint32_t tasks;     // ceil(L / 64)
  uint32_t overflow;  // L > cap
  uint32_t pad[13];
};

struct Layout {
  uint32_t* P;
  uint32_t* WF;
  uint32_t* TS;  // per-tile leaf sums (k_plan_tiles -> k_plan_scan)
  uint32_t* CV;
  uint32_t cap;
};

__host__ __device__ inline uint64_t plan_tiles(int n) { return (uint64_t(n) + kPlanThreads - 1) / kPlanThreads; }

__host__ __device__ inline uint64_t cv_offset(int n, uint64_t cap) {
  const uint64_t head = 64 + 4 * (uint64_t(n) + 1) + 4 * (cap / 64 + 2) + 4 * plan_tiles(n);
  return (head + 255) & ~uint64_t(255);
}

__host__ __device__ inline Layout layout(uint8_t* s, int n, uint32_t cap) {
  Layout l;
  l.P = reinterpret_cast<uint32_t*>(s + 64);
  l.WF = l.P + n + 1;
  l.TS = l.WF + cap / 64 + 2;
  l.CV = reinterpret_cast<uint32_t*>(s + cv_offset(n, cap));
  l.cap = cap;
  return l;
}

// Descriptor sources: the bytes + length of message c, or bad (hashed as described per source).
struct ChunkSrc {  // placed Xet chunks (k_hash_chunks semantics: a bad descriptor hashes as empty)
  const ZgChunk* chunks;
  const uint8_t* buf;
  uint64_t dst_n;
  static constexpr bool kBadIsFF = false;
  static constexpr bool kPlace = false;
  __device__ __forceinline__ void get(int c, const uint8_t*& p, uint32_t& len, bool& bad) const {
    uint64_t off = chunks[c].dst;
    len = chunks[c].ulen;
    bad = false;
    if (off + len > dst_n || len > kMaxChunk) off = 0, len = 0;
    p = buf + off;
  }
};

struct RangeSrc {  // raw (offset, len) messages (k_hash_ranges semantics: > 128 KiB -> all-ones hash)
  const uint64_t* offs;
  const uint32_t* lens;
  const uint8_t* buf;
  static constexpr bool kBadIsFF = true;
  static constexpr bool kPlace = false;
  __device__ __forceinline__ void get(int c, const uint8_t*& p, uint32_t& len, bool& bad) const {
    uint64_t off = offs[c];
    len = lens[c];
    bad = len > kMaxChunk;
    if (bad) off = 0, len = 0;
    p = buf + off;
  }
};

// Fused place + hash of one ingest launch (K3a + K1 in one pass): uncompressed (scheme 0) chunks
// are still in the staging buffer; each leaf wave first copies the raw bytes of its 64 leaves
// staging -> arena (wave_copy: 16-byte aligned stores, coalesced), then hashes them from staging,
// whose lines the copy just pulled into L2.  Compressed chunks were decoded into the arena by the
// LZ4 kernel before this launch and are hashed from there.  The arena is written once and never
// read back, where place-then-hash read it again (round 2: k_place_raw 28 % + k_hash_leaves 22 % of
// the pull's kernel time, profiles/bench70b_n1_kernels_r2c.md).
//
// A raw chunk's hash therefore covers the staging bytes the same wave just stored into the arena
// (the copy is exercised against the source bytes, misaligned both sides, by
// tests/test_gpu_kernels.py::test_fused_ingest_places_exact_bytes), and receivers of the swarm
// exchange re-hash what landed in their own arena.  A descriptor that fails its bounds check is not
// placed, is hashed over its planned leaves with no bytes in them (never its real hash, so its file's
// Merkle check fails) and is reported in the error word as ZG_ERR_RANGE at its chunk index, like the
// unfused k_place_raw did.
struct PlaceSrc {
  const ZgChunk* chunks;
  const uint8_t* src;
  uint64_t src_n;
  uint8_t* dst;
  uint64_t dst_n;
  unsigned long long* err;
  int skip_compressed = 0;  // the LZ4 decoder already hashed the compressed chunks (zg_lz4_decode_ingest)
  static constexpr bool kBadIsFF = false;
  static constexpr bool kPlace = true;
  __device__ __forceinline__ bool raw_ok(const ZgChunk& ch) const {
    return ch.src + ch.ulen <= src_n && ch.dst + ch.ulen <= dst_n && ch.ulen <= kMaxChunk;
  }
  __device__ __forceinline__ void get(int c, const uint8_t*& p, uint32_t& len, bool& bad) const {
    const ZgChunk ch = chunks[c];
    len = ch.ulen;
    if (ch.scheme == 0) {
      bad = !raw_ok(ch);
      if (bad) len = 0;
      p = src + (len ? ch.src : 0);
    } else {
      bad = ch.dst + len > dst_n || len > kMaxChunk;
      if (bad) len = 0;
      p = dst + (len ? ch.dst : 0);
    }
  }
  __device__ __forceinline__ void report(int c) const {
    if (err) atomicCAS(err, 0ull, (static_cast<unsigned long long>(ZG_ERR_RANGE) << 32) | uint32_t(c));
  }
};

template <class Src>
__device__ __forceinline__ uint32_t n_leaves(const Src& s, int c) {
  uint32_t len;
  if constexpr (Src::kPlace) {
    // the plan needs only the size: one 4-byte load instead of the 32-byte record.  A record that later fails its bounds check in get() hashes
    // as empty leaves, so its chunk hash -- and the file's Merkle check -- fails as it should.
    len = s.chunks[c].ulen;
    if (len > kMaxChunk) len = 0;
    // a chunk with no leaves gets no hash written at all (k_hash_tree skips it)
    if (s.skip_compressed && s.chunks[c].scheme != 0) return 0u;
  } else {
    const uint8_t* p;
    bool bad;
    s.get(c, p, len, bad);
  }
  return len == 0 ? 1u : (len + 1023u) >> 10;
}

__device__ __forceinline__ void store8(uint32_t* d, const uint32_t v[8]) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  reinterpret_cast<u4*>(d)[0] = u4{v[0], v[1], v[2], v[3]};
  reinterpret_cast<u4*>(d)[1] = u4{v[4], v[5], v[6], v[7]};
}

__device__ __forceinline__ void load8w(const uint32_t* s, uint32_t v[8]) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const u4 a = reinterpret_cast<const u4*>(s)[0], b = reinterpret_cast<const u4*>(s)[1];
  v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
}

__device__ __forceinline__ const zg::Key8& key_of(int key_mode) {
  return key_mode == 0 ? zg::kDataKeyW : key_mode == 1 ? zg::kNodeKeyW : key_mode == 2 ? zg::kIVW : zg::kZeroW;
}

// The plan is two chip-wide launches (round 2 ran it as one 1024-thread workgroup on a single CU,
// 18-21 us per 16k chunks, latency-bound): k_plan_tiles sums the leaves of each 1024-chunk tile,
// k_plan_scan gives every tile its base (sum of the tile sums before it, at most a few hundred
// values read by every block) and scans the tile locally.  Neither needs inter-workgroup sync.
template <class Src>
__global__ void __launch_bounds__(kPlanThreads) k_plan_tiles(Src s, int n, uint8_t* scratch, uint32_t cap) {
  __shared__ uint32_t red[kPlanThreads / kWave];
  const Layout l = layout(scratch, n, cap);
  const int t = threadIdx.x, c = blockIdx.x * kPlanThreads + t;
  const uint32_t incl = zwv::scan_add(c < n ? n_leaves(s, c) : 0u);
  if ((t & (kWave - 1)) == kWave - 1) red[t >> 6] = incl;
  __syncthreads();
  if (t == 0) {
    uint32_t sum = 0;
#pragma unroll
    for (int w = 0; w < kPlanThreads / kWave; ++w) sum += red[w];
    l.TS[blockIdx.x] = sum;
  }
}

template <class Src>
__global__ void __launch_bounds__(kPlanThreads) k_plan_scan(Src s, int n, uint8_t* scratch, uint32_t cap) {
  constexpr int W = kPlanThreads / kWave;
  __shared__ uint32_t part[W], red_before[W], red_all[W];
  const Layout l = layout(scratch, n, cap);
  const int t = threadIdx.x, wid = t >> 6, k = blockIdx.x, tiles = gridDim.x;
  // this tile's base and the grand total L from the per-tile sums
  uint32_t before = 0, all = 0;
  for (int j = t; j < tiles; j += kPlanThreads) {
    const uint32_t x = l.TS[j];
    before += j < k ? x : 0u;
    all += x;
  }
  const int c = k * kPlanThreads + t;
  const uint32_t v = c < n ? n_leaves(s, c) : 0u;
  const uint32_t incl = zwv::scan_add(v);
  const uint32_t wb = zwv::scan_add(before), wa = zwv::scan_add(all);
  if ((t & (kWave - 1)) == kWave - 1) part[wid] = incl, red_before[wid] = wb, red_all[wid] = wa;
  __syncthreads();
  uint32_t base = 0, L = 0, wave_off = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    base += red_before[w];
    L += red_all[w];
    wave_off += w < wid ? part[w] : 0u;
  }
  const bool overflow = L > cap;
  const uint32_t run = base + wave_off + incl - v;  // P[c] = first leaf of chunk c
  if (c < n) {
    l.P[c] = run;
    // WF[task] = chunk owning leaf 64 task: every chunk marks the task starts inside [run, run + v)
    if (!overflow)
      for (uint32_t g = (run + 63u) & ~63u; g < run + v; g += 64) l.WF[g >> 6] = uint32_t(c);
  }
  if (k == tiles - 1 && t == 0) {
    l.P[n] = L;
    PlanHdr* h = reinterpret_cast<PlanHdr*>(scratch);
    h->leaves = overflow ? 0u : L;
    h->tasks = overflow ? 0u : (L + 63u) >> 6;
    h->overflow = overflow ? 1u : 0u;
  }
}

// The raw bytes of wave task `task` (leaves 64 task .. 64 task + 63, chunks lo_c..hi_c) go
// staging -> arena; wave-uniform loop over the (at most ~9) chunks the task touches.
__device__ __forceinline__ void place_task(const PlaceSrc& s, const Layout& l, uint32_t task, int lo_c, int hi_c,
                                           uint32_t lane) {
  const uint32_t g0 = task * kWave, g1 = g0 + kWave;
  for (int c = lo_c; c <= hi_c; ++c) {
    const ZgChunk ch = s.chunks[c];
    if (__builtin_amdgcn_readfirstlane(ch.scheme) != 0 || !s.raw_ok(ch)) continue;
    const uint32_t p0 = __builtin_amdgcn_readfirstlane(l.P[c]), p1 = __builtin_amdgcn_readfirstlane(l.P[c + 1]);
    const uint32_t a = max(p0, g0) - p0, b = min(p1, g1) - p0;  // leaf range of this chunk in the task
    if (a >= b) continue;
    const uint64_t lo = uint64_t(a) << 10, hi = min(uint64_t(b) << 10, uint64_t(ch.ulen));
    if (lo < hi) zwv::wave_copy(s.dst + ch.dst + lo, s.src + ch.src + lo, hi - lo, lane);
  }
}

template <class Src>
__global__ void __launch_bounds__(256) k_hash_leaves(Src s, int n, int key_mode, uint8_t* scratch, uint32_t cap,
                                                     uint8_t* __restrict__ out, uint64_t* __restrict__ sizes) {
  const Layout l = layout(scratch, n, cap);
  const PlanHdr* h = reinterpret_cast<const PlanHdr*>(scratch);
  const uint32_t T = __builtin_amdgcn_readfirstlane(h->tasks);
  const uint32_t L = __builtin_amdgcn_readfirstlane(h->leaves);
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  const zg::Key8& key = key_of(key_mode);
  const uint32_t mode = key_mode == 2 ? 0u : zg::KEYED_HASH;
  for (uint32_t task = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6));
       task < T; task += waves) {
    const uint32_t g = task * kWave + lane;
    // the owner of leaf g lies in [WF[task], WF[task + 1]]: binary search of P over that range
    int lo = int(__builtin_amdgcn_readfirstlane(l.WF[task]));
    int hi = task + 1 < T ? int(__builtin_amdgcn_readfirstlane(l.WF[task + 1])) : n - 1;
    if constexpr (Src::kPlace) place_task(s, l, task, lo, hi, lane);
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (l.P[mid] <= g) lo = mid;
      else hi = mid - 1;
    }
    if (g >= L) continue;
    const int c = lo;
    const uint32_t b = g - l.P[c];
    const uint32_t nb = l.P[c + 1] - l.P[c];
    const uint8_t* p;
    uint32_t len;
    bool bad;
    s.get(c, p, len, bad);
    const uint32_t seg = len > (b << 10) ? min(len - (b << 10), 1024u) : 0u;
    uint32_t cv[8];
    if constexpr (Src::kPlace) {
      if (bad && b == 0) s.report(c);  // one report per bad descriptor (its first leaf's lane)
    }
    zg::hash_leaf(p + (uint64_t(b) << 10), seg, b, key, mode, nb == 1, cv);
    if (nb == 1) {
      if (Src::kBadIsFF && bad) {
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[i] = 0xFFFFFFFFu;
      }
      store8(reinterpret_cast<uint32_t*>(out + 32 * uint64_t(c)), cv);
    } else {
      store8(l.CV + 8 * uint64_t(g), cv);
    }
    if (sizes && b == 0) sizes[c] = len;
  }
}

// kTreeG chunks per wave, 4 independent waves per block, nodes in place in the scratch CV array
// (an LDS copy of the group's CVs was slower: 32 KiB per wave cut residency to 5 waves per CU, and
// this kernel is latency-bound).  Level s+1 reads what level s stored: a workgroup-scope
// release/acquire between levels orders them (one CU, so its vector L1 sees the wave's own stores).
__global__ void __launch_bounds__(256) k_hash_tree(int n, int key_mode, uint8_t* scratch, uint32_t cap,
                                                   uint8_t* __restrict__ out) {
  const Layout l = layout(scratch, n, cap);
  const PlanHdr* h = reinterpret_cast<const PlanHdr*>(scratch);
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const int c0 = __builtin_amdgcn_readfirstlane((blockIdx.x * (blockDim.x / kWave) + (threadIdx.x >> 6)) * kTreeG);
  if (c0 >= n) return;
  if (__builtin_amdgcn_readfirstlane(h->overflow)) {  // undersized scratch: nothing verifies
    if (c0 + int(lane >> 3) < n) reinterpret_cast<uint32_t*>(out + 32 * uint64_t(c0))[lane] = 0xFFFFFFFFu;
    return;
  }
  const zg::Key8& key = key_of(key_mode);
  const uint32_t mode = key_mode == 2 ? 0u : zg::KEYED_HASH;
  // uniform per-chunk state: CV base (leaf offset) and live node count (1 = done / one-leaf chunk)
  const uint32_t pv = l.P[min(c0 + int(lane), n)];
  uint32_t base[kTreeG], m[kTreeG];
#pragma unroll
  for (int i = 0; i < kTreeG; ++i) {
    base[i] = __builtin_amdgcn_readlane(pv, i);
    const uint32_t nxt = __builtin_amdgcn_readlane(pv, i + 1);
    m[i] = c0 + i < n ? nxt - base[i] : 1u;
  }
  while (true) {
    uint32_t tp[kTreeG + 1];
    tp[0] = 0;
#pragma unroll
    for (int i = 0; i < kTreeG; ++i) tp[i + 1] = tp[i] + (m[i] >= 2 ? (m[i] + 1) >> 1 : 0u);
    const uint32_t tasks = tp[kTreeG];
    if (tasks == 0) break;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (uint32_t t0 = 0; t0 < tasks; t0 += kWave) {
      const uint32_t t = t0 + lane;
      if (t < tasks) {
        uint32_t mi = m[0], bi = base[0], ti = 0;
        int ci = 0;
#pragma unroll
        for (int i = 1; i < kTreeG; ++i)
          if (t >= tp[i]) mi = m[i], bi = base[i], ti = tp[i], ci = i;
        const uint32_t j = t - ti, pairs = mi >> 1;
        const bool pair = j < pairs;  // else: the odd last node moves up unchanged
        uint32_t* nodes = l.CV + 8 * uint64_t(bi);
        uint32_t lft[8], rgt[8], o[8];
        load8w(nodes + 8 * (2 * j), lft);
        load8w(nodes + 8 * (pair ? 2 * j + 1 : 2 * j), rgt);
        zg::parent_cv(lft, rgt, key, mode, mi == 2, o);
        if (!pair) {
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = lft[k];
        }
        if (mi == 2) store8(reinterpret_cast<uint32_t*>(out + 32 * uint64_t(c0 + ci)), o);
        else store8(nodes + 8 * j, o);
      }
    }
#pragma unroll
    for (int i = 0; i < kTreeG; ++i) m[i] = m[i] >= 2 ? (m[i] + 1) >> 1 : m[i];
  }
}

uint32_t cap_of(int n, size_t bytes) {
  // largest cap with cv_offset(n, cap) + 32 cap <= bytes
  if (bytes < 1024) return 0;
  uint64_t cap = bytes / 32;
  while (cap > 0 && cv_offset(n, cap) + 32 * cap > bytes) {
    const uint64_t over = cv_offset(n, cap) + 32 * cap - bytes;
    cap -= over / 32 + 1;
  }
  return cap > 0xFFFFFFF0ull ? 0xFFFFFFF0u : uint32_t(cap);
}

template <class Src>
hipError_t launch_flat(Src s, int n, int key_mode, uint8_t* out, uint64_t* sizes, uint8_t* scratch,
                       size_t scratch_bytes, hipStream_t stream) {
  const uint32_t cap = cap_of(n, scratch_bytes);
  if (cap == 0) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  const uint32_t tiles = uint32_t(plan_tiles(n));
  hipLaunchKernelGGL((k_plan_tiles<Src>), dim3(tiles), dim3(kPlanThreads), 0, stream, s, n, scratch, cap);
  hipLaunchKernelGGL((k_plan_scan<Src>), dim3(tiles), dim3(kPlanThreads), 0, stream, s, n, scratch, cap);
  const uint64_t task_bound = (uint64_t(cap) + 63) / 64;
  const uint32_t waves = uint32_t(task_bound < kLeafMaxWaves ? task_bound : kLeafMaxWaves);
  hipLaunchKernelGGL((k_hash_leaves<Src>), dim3((waves + 3) / 4), dim3(256), 0, stream, s, n, key_mode, scratch, cap,
                     out, sizes);
  const int groups = (n + kTreeG - 1) / kTreeG;
  hipLaunchKernelGGL(k_hash_tree, dim3((groups + 3) / 4), dim3(256), 0, stream, n, key_mode, scratch, cap, out);
  return hipGetLastError();
}

}  // namespace

extern "C" {

size_t zg_hash_scratch_bytes(int n, uint64_t total_bytes) {
  if (n <= 0) return 0;
  const uint64_t cap = total_bytes / 1024 + uint64_t(n) + 64;
  return size_t(cv_offset(n, cap) + 32 * cap);
}

size_t zg_ingest_scratch_bytes(int n, uint64_t total_bytes) {
  // an ingest launch's scratch serves its BG4 decode staging first, then the place/hash pass
  const size_t hash = zg_hash_scratch_bytes(n, total_bytes), stage = zg_lz4_stage_bytes(n);
  return hash > stage ? hash : stage;
}

hipError_t zg_hash_chunks_flat(const uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks, int n_chunks,
                               uint8_t* hashes, uint64_t* sizes, uint8_t* scratch, size_t scratch_bytes,
                               hipStream_t stream) {
  return launch_flat(ChunkSrc{chunks, dst, dst_n}, n_chunks, 0, hashes, sizes, scratch, scratch_bytes, stream);
}

hipError_t zg_place_hash_flat(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                              int n_chunks, unsigned long long* err, uint8_t* hashes, uint64_t* sizes, uint8_t* scratch,
                              size_t scratch_bytes, hipStream_t stream) {
  return launch_flat(PlaceSrc{chunks, src, src_n, dst, dst_n, err}, n_chunks, 0, hashes, sizes, scratch, scratch_bytes,
                     stream);
}

hipError_t zg_place_hash_flat_raw(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                  const ZgChunk* chunks, int n_chunks, unsigned long long* err, uint8_t* hashes,
                                  uint64_t* sizes, uint8_t* scratch, size_t scratch_bytes, hipStream_t stream) {
  return launch_flat(PlaceSrc{chunks, src, src_n, dst, dst_n, err, 1}, n_chunks, 0, hashes, sizes, scratch,
                     scratch_bytes, stream);
}

hipError_t zg_hash_ranges_flat(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lens, int n,
                               uint8_t* hashes, int key_mode, uint8_t* scratch, size_t scratch_bytes,
                               hipStream_t stream) {
  return launch_flat(RangeSrc{offsets, lens, buf}, n, key_mode, hashes, nullptr, scratch, scratch_bytes, stream);
}

}  // extern "C"
