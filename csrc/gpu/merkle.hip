// K2: Xet Merkle aggregation on the GPU, per tree (file or xorb).  Levels 1 and 2 (~15/16 of the
// node hashing) run across the whole chip: group boundaries with one 1024-thread workgroup per
// tree, node hashes with many workgroups per tree; levels 3+ with one workgroup per tree.  Per level: (1) cut flags u64(hash[24:32]) % 4 == 0 into a bitmask, (2) group
// boundaries (first flagged child at index >= 2, at most 9 children) by a parallel chain walk,
// (3) "{xet_hex} : {size}\n" lines of each group hashed with the INTERNAL_NODE key.  The root
// optionally becomes the file hash (BLAKE3 keyed with the all-zero salt).  Host oracle:
// csrc/core/xet_hash.cpp.
#include <hip/hip_runtime.h>

#include "blake3_dev.h"
#include "zgpu.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kHashThreads = 512;  // k_merkle threads that hash nodes (128-byte LDS ring each)
// Rings sit kRingStride dwords apart: 33 (odd) puts the 64 lanes of a wave in 64 different LDS
// banks.  With 32 every lane's ring started in the same bank, and rocprof counted 9.9 bank
// conflicts per LDS access in k_merkle_spread (profiles/r5/pmc_table_gpubench256_r5h.md).
constexpr int kRingStride = 33;
constexpr uint32_t kLdsFlagWords = 4096;  // cut flags of levels with <= 131072 nodes live in LDS

struct JobScratch {
  uint32_t* hdr;     // [0] = groups of level 1 (written by k_merkle_starts)
  uint8_t* hash_a;   // [n][32]
  uint64_t* size_a;  // [n]
  uint8_t* hash_b;
  uint64_t* size_b;
  uint32_t* flags;   // [ceil(n/32)]
  uint32_t* starts;  // [n/2 + 2]
};

__host__ __device__ inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

__host__ __device__ inline uint64_t job_scratch_bytes(uint64_t n) {
  const uint64_t nn = n < 2 ? 2 : n;
  return 256 + align_up(nn * 32, 256) * 2 + align_up(nn * 8, 256) * 2 + align_up((nn + 31) / 32 * 4, 256) +
         align_up((nn / 2 + 4) * 4, 256);
}

__device__ inline JobScratch carve(uint8_t* base, uint64_t n) {
  const uint64_t nn = n < 2 ? 2 : n;
  JobScratch s;
  uint8_t* p = base;
  s.hdr = reinterpret_cast<uint32_t*>(p);
  p += 256;
  s.hash_a = p;
  p += align_up(nn * 32, 256);
  s.hash_b = p;
  p += align_up(nn * 32, 256);
  s.size_a = reinterpret_cast<uint64_t*>(p);
  p += align_up(nn * 8, 256);
  s.size_b = reinterpret_cast<uint64_t*>(p);
  p += align_up(nn * 8, 256);
  s.flags = reinterpret_cast<uint32_t*>(p);
  p += align_up((nn + 31) / 32 * 4, 256);
  s.starts = reinterpret_cast<uint32_t*>(p);
  return s;
}

// Decimal digits of v, most significant first, as packed nibbles (digit i = nibble i of lo:hi)
// -- division by the constant 10 only (mul-high), 32-bit while the value fits.
__device__ inline uint32_t dec_digits(uint64_t v, uint64_t& lo, uint64_t& hi) {
  uint32_t nd = 0;
  lo = hi = 0;
  auto push = [&](uint32_t d) {
    hi = (hi << 4) | (lo >> 60);
    lo = (lo << 4) | d;
    ++nd;
  };
  while (v >> 32) {
    const uint64_t q = v / 10u;
    push(uint32_t(v - q * 10u));
    v = q;
  }
  uint32_t w = uint32_t(v);
  do {
    const uint32_t q = w / 10u;
    push(w - q * 10u);
    w = q;
  } while (w);
  return nd;
}

__device__ inline uint32_t ndigits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10000) v /= 10000, d += 4;
  while (v >= 10) v /= 10, ++d;
  return d;
}

// One internal node: keyed BLAKE3 (INTERNAL_NODE key) of the lines "{xet_hex} : {size}\n" of
// children [a, b) -- a single BLAKE3 chunk (<= 9 lines < 1 KiB), so its length is known up front
// for the CHUNK_END/ROOT flags.  SIMT layout: the bytes go into a private 128-byte LDS ring and
// full blocks are compressed only at two points per line (after the 64 hex digits, which always
// complete a block, and after the " : size\n" tail), so a wave's lanes compress together instead
// of each lane hitting its block boundary at a different byte (which made the wave run ~8x more
// compressions than it needed).
__device__ void hash_node(const uint8_t* cur_h, const uint64_t* cur_s, uint32_t a, uint32_t b, uint8_t* ring,
                          uint8_t* dst_h, uint64_t* dst_s) {
  uint32_t msg_len = 0;
  for (uint32_t j = a; j < b; ++j) msg_len += 68 + ndigits(cur_s[j]);
  uint32_t cv[8];
  zg::load_key(cv, zg::kNodeKeyW);
  uint32_t pos = 0, done = 0;  // bytes written / bytes compressed
  uint64_t total = 0;
  auto flush = [&]() {  // compress the block at `done` once complete, unless it is the last one
    if (pos - done >= 64 && done + 64 < msg_len) {
      uint32_t m[16];
      const uint32_t* w = reinterpret_cast<const uint32_t*>(ring + (done & 127));
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = w[i];
      zg::compress(cv, m, 0, 64, zg::KEYED_HASH | (done == 0 ? zg::CHUNK_START : 0u));
      done += 64;
    }
  };
#pragma unroll 1
  for (uint32_t j = a; j < b; ++j) {
    const uint64_t* hw = reinterpret_cast<const uint64_t*>(cur_h + 32 * size_t(j));
    const uint64_t v0 = hw[0], v1 = hw[1], v2 = hw[2], v3 = hw[3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t v = q == 0 ? v0 : q == 1 ? v1 : q == 2 ? v2 : v3;
#pragma unroll
      for (int d = 60; d >= 0; d -= 4) {
        const uint32_t nib = uint32_t(v >> d) & 15u;
        ring[pos++ & 127] = uint8_t(nib < 10 ? '0' + nib : 'a' + nib - 10);
      }
    }
    flush();
    ring[pos++ & 127] = ' ';
    ring[pos++ & 127] = ':';
    ring[pos++ & 127] = ' ';
    const uint64_t sz = cur_s[j];
    total += sz;
    uint64_t lo, hi;
    const uint32_t nd = dec_digits(sz, lo, hi);
    for (uint32_t i = 0; i < nd; ++i)
      ring[pos++ & 127] = uint8_t('0' + uint32_t((i < 16 ? lo >> (4 * i) : hi >> (4 * (i - 16))) & 15u));
    ring[pos++ & 127] = '\n';
    flush();
  }
  for (uint32_t i = pos; i < done + 64; ++i) ring[i & 127] = 0;
  uint32_t m[16];
  const uint32_t* w = reinterpret_cast<const uint32_t*>(ring + (done & 127));
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = w[i];
  zg::compress(cv, m, 0, msg_len - done,
               zg::KEYED_HASH | zg::CHUNK_END | zg::ROOT | (done == 0 ? zg::CHUNK_START : 0u));
  uint32_t* dst = reinterpret_cast<uint32_t*>(dst_h);
  for (int k = 0; k < 8; ++k) dst[k] = cv[k];
  *dst_s = total;
}

struct LevelLds {
  uint32_t ngroups;
  uint8_t exit[kThreads][9];
  uint8_t entry[kThreads];
  uint32_t scan[kThreads];
  uint32_t flags[kLdsFlagWords];
};

// Group boundaries of one level (block-wide): cut flags u64(hash[24:32]) % 4 == 0, then the chain
// p -> p + cut(p) (close after the first flagged child at index >= 2, at most 9 children) computed
// in parallel: thread t owns positions [t*B, (t+1)*B); a group that starts before a block ends at
// most 8 positions into it, so (A) each thread maps its block's 9 possible entry offsets to exit
// offsets, (B) a scan of the map composition gives every block its true entry, (C) each thread
// re-walks from its entry counting starts, and after a block scan (D) writes them.  O(n/T)
// dependent steps per thread.
// Returns the group count; s.starts[0..ng] holds the boundaries.
__device__ uint32_t level_starts(const uint8_t* cur_h, uint64_t n, const JobScratch& s, LevelLds& L) {
  const uint32_t tid = threadIdx.x;
  const uint64_t nwords = (n + 31) / 32;
  for (uint64_t i = tid; i < nwords; i += kThreads) {
    // u64 little-endian of hash bytes 24..32; % 4 only needs the low byte.  A full word's 32 loads
    // share one base address (immediate offsets) and are all in flight together.
    const uint32_t* w6 = reinterpret_cast<const uint32_t*>(cur_h + 32 * 32 * i) + 6;
    uint32_t word = 0;
    if (32 * i + 32 <= n) {
      uint32_t low[32];
#pragma unroll
      for (uint32_t b = 0; b < 32; ++b) low[b] = w6[8 * b];
#pragma unroll
      for (uint32_t b = 0; b < 32; ++b) word |= (low[b] & 3u) == 0 ? 1u << b : 0u;
    } else {
      for (uint32_t b = 0; 32 * i + b < n; ++b) word |= (w6[8 * b] & 3u) == 0 ? 1u << b : 0u;
    }
    if (nwords <= kLdsFlagWords) L.flags[i] = word;
    else s.flags[i] = word;
  }
  __syncthreads();
  const uint32_t* flags = nwords <= kLdsFlagWords ? L.flags : s.flags;
  const uint64_t B = (n + kThreads - 1) / kThreads;
  const uint64_t lo = uint64_t(tid) * B;
  const uint64_t hi = lo + B < n ? lo + B : n;
  auto cut_at = [&](uint64_t p) -> uint64_t {
    const uint64_t rem = n - p;
    if (rem <= 2) return rem;
    const uint64_t end = rem < 9 ? rem : 9;
    for (uint64_t i = 2; i < end; ++i) {
      const uint64_t j = p + i;
      if ((flags[j >> 5] >> (j & 31)) & 1u) return i + 1;
    }
    return end;
  };
  if (lo < hi) {
    // entry 0 walks the whole block; every other entry walks only until its chain lands on a
    // position of entry 0's chain (chains merge within a group or two), then shares its exit
    uint64_t p0 = lo;
    while (p0 < hi) p0 += cut_at(p0);
    const uint8_t ex0 = uint8_t(p0 - hi);
    L.exit[tid][0] = ex0;
    for (uint32_t e = 1; e < 9; ++e) {
      uint64_t p = lo + e, q = lo;
      uint8_t ex = 0xFF;
      while (p < hi) {
        while (q < p) q += cut_at(q);
        if (q == p) {
          ex = ex0;
          break;
        }
        p += cut_at(p);
      }
      L.exit[tid][e] = ex != 0xFF ? ex : uint8_t(p - hi);
    }
  } else {
#pragma unroll
    for (uint32_t e = 0; e < 9; ++e) L.exit[tid][e] = uint8_t(e);  // past the end: identity map
  }
  __syncthreads();
  // Block entries: entry_t = (X_{t-1} o ... o X_0)(0) with X_t the block's entry -> exit map.
  // Inclusive scan of the map composition (Hillis-Steele, 10 steps) instead of one thread
  // chaining all 1024 blocks.
  for (uint32_t d = 1; d < uint32_t(kThreads); d <<= 1) {
    uint8_t nxt[9];
    if (tid >= d) {
#pragma unroll
      for (uint32_t e = 0; e < 9; ++e) nxt[e] = L.exit[tid][L.exit[tid - d][e]];
    }
    __syncthreads();
    if (tid >= d) {
#pragma unroll
      for (uint32_t e = 0; e < 9; ++e) L.exit[tid][e] = nxt[e];
    }
    __syncthreads();
  }
  L.entry[tid] = tid == 0 ? 0 : L.exit[tid - 1][0];
  __syncthreads();
  uint32_t cnt = 0;
  if (lo < hi) {
    for (uint64_t p = lo + L.entry[tid]; p < hi; p += cut_at(p)) ++cnt;
  }
  // block-wide exclusive scan of cnt (Hillis-Steele in LDS)
  L.scan[tid] = cnt;
  __syncthreads();
  for (uint32_t d = 1; d < uint32_t(kThreads); d <<= 1) {
    const uint32_t v = tid >= d ? L.scan[tid - d] : 0;
    __syncthreads();
    L.scan[tid] += v;
    __syncthreads();
  }
  const uint32_t base = L.scan[tid] - cnt;
  if (lo < hi) {
    uint32_t g = base;
    for (uint64_t p = lo + L.entry[tid]; p < hi; p += cut_at(p)) s.starts[g++] = uint32_t(p);
  }
  if (tid == kThreads - 1) {
    s.starts[L.scan[tid]] = uint32_t(n);
    L.ngroups = L.scan[tid];
  }
  __syncthreads();
  return L.ngroups;
}

// Levels 1 and 2 run on the whole chip: per level, group boundaries (one workgroup per tree,
// k_merkle_starts) then the node hashes spread over many workgroups per tree (k_merkle_spread).
// They hold ~15/16 of a tree's node hashing, which one workgroup per tree left on 30 CUs for a
// 30-file model.  Level L (1 or 2) reads the leaves (L = 1) or level 1 and writes hash_a/size_a
// (L = 1) or hash_b/size_b (L = 2); hdr[L - 1] = its node count.  A tree already down to one node
// is copied through, so k_merkle always continues from hash_b.
struct LevelIo {
  const uint8_t* in_h;
  const uint64_t* in_s;
  uint64_t n_in;
  uint8_t* out_h;
  uint64_t* out_s;
};

__device__ inline LevelIo level_io(const ZgMerkleJob& job, const uint8_t* leaf_hashes, const uint64_t* leaf_sizes,
                                   const JobScratch& s, int level) {
  LevelIo io;
  if (level == 1) {
    io.in_h = leaf_hashes + 32 * job.leaf_base;
    io.in_s = leaf_sizes + job.leaf_base;
    io.n_in = job.n_leaves;
    io.out_h = s.hash_a;
    io.out_s = s.size_a;
  } else {
    io.in_h = s.hash_a;
    io.in_s = s.size_a;
    io.n_in = s.hdr[0];
    io.out_h = s.hash_b;
    io.out_s = s.size_b;
  }
  return io;
}

__global__ void __launch_bounds__(kThreads) k_merkle_starts(const uint8_t* __restrict__ leaf_hashes,
                                                            const uint64_t* __restrict__ leaf_sizes,
                                                            const ZgMerkleJob* __restrict__ jobs,
                                                            uint8_t* __restrict__ scratch, uint64_t per_job, int level) {
  __shared__ LevelLds L;
  const ZgMerkleJob job = jobs[blockIdx.x];
  JobScratch s = carve(scratch + per_job * blockIdx.x, job.n_leaves);
  const LevelIo io = level_io(job, leaf_hashes, leaf_sizes, s, level);
  if (io.n_in <= 1) {
    if (threadIdx.x == 0) s.hdr[level - 1] = uint32_t(io.n_in);
    return;
  }
  const uint32_t ng = level_starts(io.in_h, io.n_in, s, L);
  if (threadIdx.x == 0) s.hdr[level - 1] = ng;
}

constexpr int kNodeThreads = 256;
__global__ void __launch_bounds__(kNodeThreads) k_merkle_spread(const uint8_t* __restrict__ leaf_hashes,
                                                                const uint64_t* __restrict__ leaf_sizes,
                                                                const ZgMerkleJob* __restrict__ jobs,
                                                                uint8_t* __restrict__ scratch, uint64_t per_job,
                                                                int level, int spread) {
  __shared__ uint32_t s_ring[kNodeThreads * kRingStride];
  const uint32_t jb = blockIdx.x / spread, part = blockIdx.x % spread;
  const ZgMerkleJob job = jobs[jb];
  JobScratch s = carve(scratch + per_job * jb, job.n_leaves);
  const LevelIo io = level_io(job, leaf_hashes, leaf_sizes, s, level);
  if (io.n_in <= 1) {  // nothing to merge: carry the single node to this level's output
    if (io.n_in == 1 && part == 0 && threadIdx.x < 8) {
      reinterpret_cast<uint32_t*>(io.out_h)[threadIdx.x] = reinterpret_cast<const uint32_t*>(io.in_h)[threadIdx.x];
      if (threadIdx.x == 0) io.out_s[0] = io.in_s[0];
    }
    return;
  }
  const uint32_t ng = s.hdr[level - 1];
  uint8_t* ring = reinterpret_cast<uint8_t*>(&s_ring[threadIdx.x * kRingStride]);
  for (uint32_t g = part * kNodeThreads + threadIdx.x; g < ng; g += uint32_t(spread) * kNodeThreads)
    hash_node(io.in_h, io.in_s, s.starts[g], s.starts[g + 1], ring, io.out_h + 32 * size_t(g), io.out_s + g);
}

// Levels 3+ (one workgroup per tree), then the root / file hash.
__global__ void __launch_bounds__(kThreads) k_merkle(const uint8_t* __restrict__ leaf_hashes,
                                                     const uint64_t* __restrict__ leaf_sizes,
                                                     const ZgMerkleJob* __restrict__ jobs, uint8_t* __restrict__ roots,
                                                     uint8_t* __restrict__ scratch, uint64_t per_job) {
  __shared__ LevelLds L;
  __shared__ uint32_t s_ring[kHashThreads * kRingStride];
  const ZgMerkleJob job = jobs[blockIdx.x];
  const uint32_t tid = threadIdx.x;
  uint8_t* out = roots + 32 * size_t(blockIdx.x);
  uint64_t n = job.n_leaves;
  if (n == 0) {
    if (tid < 32) out[tid] = 0;
    return;
  }
  JobScratch s = carve(scratch + per_job * blockIdx.x, n);
  const uint8_t* cur_h = leaf_hashes + 32 * job.leaf_base;
  const uint64_t* cur_s = leaf_sizes + job.leaf_base;
  // levels 1 and 2 were built by k_merkle_starts + k_merkle_spread (a one-node level is carried)
  n = s.hdr[1];
  cur_h = s.hash_b;
  cur_s = s.size_b;
  bool into_a = true;
  uint8_t* ring = reinterpret_cast<uint8_t*>(&s_ring[(tid % kHashThreads) * kRingStride]);
  while (n > 1) {
    const uint32_t ng = level_starts(cur_h, n, s, L);
    uint8_t* nxt_h = into_a ? s.hash_a : s.hash_b;
    uint64_t* nxt_s = into_a ? s.size_a : s.size_b;
    if (tid < kHashThreads)  // levels 3+ are small (~n/64 nodes): 512 threads with LDS rings
      for (uint32_t g = tid; g < ng; g += kHashThreads)
        hash_node(cur_h, cur_s, s.starts[g], s.starts[g + 1], ring, nxt_h + 32 * size_t(g), nxt_s + g);
    __syncthreads();
    cur_h = nxt_h;
    cur_s = nxt_s;
    into_a = !into_a;
    n = ng;
  }
  if (tid == 0) {
    uint32_t cv[8];
    if (job.want_file_hash) {
      zg::hash_chunk(cur_h, 32, 0, zg::kZeroW, zg::KEYED_HASH, true, cv);
    } else {
      const uint32_t* r = reinterpret_cast<const uint32_t*>(cur_h);
      for (int k = 0; k < 8; ++k) cv[k] = r[k];
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(out);
    for (int k = 0; k < 8; ++k) o[k] = cv[k];
  }
}

}  // namespace

extern "C" {

size_t zg_merkle_scratch_bytes(uint64_t max_leaves_per_job, int n_jobs) {
  return size_t(job_scratch_bytes(max_leaves_per_job)) * size_t(n_jobs > 0 ? n_jobs : 1) + 4096;
}

hipError_t zg_merkle(const uint8_t* leaf_hashes, const uint64_t* leaf_sizes, const ZgMerkleJob* jobs, int n_jobs,
                     uint8_t* roots, uint8_t* scratch, uint64_t scratch_bytes, hipStream_t stream) {
  if (n_jobs <= 0) return hipSuccess;
  // Per-job scratch stride is computed by the caller-visible formula from the largest job; the
  // caller sized `scratch` with zg_merkle_scratch_bytes(max_leaves, n_jobs).
  const uint64_t per_job = (scratch_bytes - 4096) / uint64_t(n_jobs);
  const uint64_t stride = per_job / 256 * 256;
  // node-hash workgroups per tree: enough for ~2k workgroups in all, at least 8 per tree
  const int spread = n_jobs >= 256 ? 8 : (2048 + n_jobs - 1) / n_jobs;
  for (int level = 1; level <= 2; ++level) {
    hipLaunchKernelGGL(k_merkle_starts, dim3(n_jobs), dim3(kThreads), 0, stream, leaf_hashes, leaf_sizes, jobs, scratch,
                       stride, level);
    hipLaunchKernelGGL(k_merkle_spread, dim3(n_jobs * spread), dim3(kNodeThreads), 0, stream, leaf_hashes, leaf_sizes,
                       jobs, scratch, stride, level, spread);
  }
  hipLaunchKernelGGL(k_merkle, dim3(n_jobs), dim3(kThreads), 0, stream, leaf_hashes, leaf_sizes, jobs, roots, scratch,
                     stride);
  return hipGetLastError();
}

}  // extern "C"
