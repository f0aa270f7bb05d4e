// K2: Xet Merkle aggregation on the GPU.  One 256-thread workgroup per tree (file or xorb).
// Per level: (1) all threads compute the cut flags u64(hash[24:32]) % 4 == 0 into a bitmask,
// (2) one lane walks the bitmask to place group boundaries (next_merge_cut: first flagged child
// at index >= 2, at most 9 children), (3) all threads format "{xet_hex} : {size}\n" lines and
// hash their groups with the INTERNAL_NODE key.  The root optionally becomes the file hash
// (BLAKE3 keyed with the all-zero salt).  Host oracle: csrc/core/xet_hash.cpp.
#include <hip/hip_runtime.h>

#include "blake3_dev.h"
#include "zgpu.h"

namespace {

constexpr int kThreads = 1024;
constexpr uint32_t kMsgBytes = 1024;
constexpr uint32_t kLdsFlagWords = 4096;  // cut flags of levels with <= 131072 nodes live in LDS  // 9 children * (64 + 3 + 20 + 1) = 792 < 1024

struct JobScratch {
  uint8_t* hash_a;   // [n][32]
  uint64_t* size_a;  // [n]
  uint8_t* hash_b;
  uint64_t* size_b;
  uint32_t* flags;   // [ceil(n/32)]
  uint32_t* starts;  // [n/2 + 2]
  uint8_t* msg;      // [kThreads][kMsgBytes]
};

__host__ __device__ inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

__host__ __device__ inline uint64_t job_scratch_bytes(uint64_t n) {
  const uint64_t nn = n < 2 ? 2 : n;
  return align_up(nn * 32, 256) * 2 + align_up(nn * 8, 256) * 2 + align_up((nn + 31) / 32 * 4, 256) +
         align_up((nn / 2 + 4) * 4, 256) + uint64_t(kThreads) * kMsgBytes;
}

__device__ inline JobScratch carve(uint8_t* base, uint64_t n) {
  const uint64_t nn = n < 2 ? 2 : n;
  JobScratch s;
  uint8_t* p = base;
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
  p += align_up((nn / 2 + 4) * 4, 256);
  s.msg = p;
  return s;
}

__device__ inline uint32_t ndigits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10) {
    v /= 10;
    ++d;
  }
  return d;
}

__device__ inline uint32_t put_line(uint8_t* m, uint32_t pos, const uint8_t* h, uint64_t size) {
  const char* hex = "0123456789abcdef";
  for (int w = 0; w < 4; ++w) {
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) v |= uint64_t(h[8 * w + b]) << (8 * b);
    for (int d = 15; d >= 0; --d) {
      m[pos + 16 * w + d] = uint8_t(hex[v & 15]);
      v >>= 4;
    }
  }
  pos += 64;
  m[pos++] = ' ';
  m[pos++] = ':';
  m[pos++] = ' ';
  char digits[24];
  int nd = 0;
  do {
    digits[nd++] = char('0' + size % 10);
    size /= 10;
  } while (size);
  while (nd) m[pos++] = uint8_t(digits[--nd]);
  m[pos++] = '\n';
  return pos;
}

__global__ void __launch_bounds__(kThreads) k_merkle(const uint8_t* __restrict__ leaf_hashes,
                                                     const uint64_t* __restrict__ leaf_sizes,
                                                     const ZgMerkleJob* __restrict__ jobs, uint8_t* __restrict__ roots,
                                                     uint8_t* __restrict__ scratch, uint64_t per_job) {
  __shared__ uint32_t s_ngroups;
  __shared__ uint8_t s_exit[kThreads][9];
  __shared__ uint8_t s_entry[kThreads];
  __shared__ uint32_t s_scan[kThreads];
  __shared__ uint32_t s_blk[kThreads * 17];
  __shared__ uint32_t s_flags[kLdsFlagWords];
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
  bool into_a = true;
  while (n > 1) {
    const uint64_t nwords = (n + 31) / 32;
    for (uint64_t i = tid; i < nwords; i += kThreads) {
      uint32_t word = 0;
      for (uint32_t b = 0; b < 32; ++b) {
        const uint64_t j = 32 * i + b;
        if (j < n) {
          const uint32_t* hw = reinterpret_cast<const uint32_t*>(cur_h + 32 * j);
          // u64 little-endian of bytes 24..32; % 4 only needs the low byte.
          if ((hw[6] & 3u) == 0) word |= 1u << b;
        }
      }
      if (nwords <= kLdsFlagWords) s_flags[i] = word;
      else s.flags[i] = word;
    }
    __syncthreads();
    const uint32_t* flags = nwords <= kLdsFlagWords ? s_flags : s.flags;
    // Group boundaries in parallel.  The rule (close after the first flagged child at index >= 2,
    // at most 9 children) is a chain p -> p + cut(p); thread t owns positions [t*B, (t+1)*B).  A
    // group that starts before a block ends at most 8 positions into it, so (A) each thread walks
    // its block from all 9 possible entry offsets, (B) one thread chains the 1024 exit offsets,
    // (C) each thread re-walks from its true entry counting starts, and after a block scan (D)
    // writes them.  O(n/T) dependent steps per thread instead of O(n) on one thread.
    {
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
        for (uint32_t e = 0; e < 9; ++e) {
          uint64_t p = lo + e;
          while (p < hi) p += cut_at(p);
          s_exit[tid][e] = uint8_t(p >= hi ? p - hi : 0);
        }
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t entry = 0;
        for (uint32_t t = 0; t < uint32_t(kThreads) && uint64_t(t) * B < n; ++t) {
          s_entry[t] = uint8_t(entry);
          entry = s_exit[t][entry];
        }
      }
      __syncthreads();
      uint32_t cnt = 0;
      if (lo < hi) {
        for (uint64_t p = lo + s_entry[tid]; p < hi; p += cut_at(p)) ++cnt;
      }
      // block-wide exclusive scan of cnt (Hillis-Steele in LDS)
      s_scan[tid] = cnt;
      __syncthreads();
      for (uint32_t d = 1; d < uint32_t(kThreads); d <<= 1) {
        const uint32_t v = tid >= d ? s_scan[tid - d] : 0;
        __syncthreads();
        s_scan[tid] += v;
        __syncthreads();
      }
      const uint32_t base = s_scan[tid] - cnt;
      if (lo < hi) {
        uint32_t g = base;
        for (uint64_t p = lo + s_entry[tid]; p < hi; p += cut_at(p)) s.starts[g++] = uint32_t(p);
      }
      if (tid == kThreads - 1) {
        s.starts[s_scan[tid]] = uint32_t(n);
        s_ngroups = s_scan[tid];
      }
    }
    __syncthreads();
    const uint32_t ng = s_ngroups;
    uint8_t* nxt_h = into_a ? s.hash_a : s.hash_b;
    uint64_t* nxt_s = into_a ? s.size_a : s.size_b;
    // Node hashes: each thread streams its group's lines "{xet_hex} : {size}\n" byte by byte into
    // a private 64-byte LDS block (stride 68 B: conflict-free banks) and compresses every full
    // block; the message (<= 9 lines, < 1 KiB) is a single BLAKE3 chunk, so its total length is
    // known up front for the CHUNK_END/ROOT flags.
    uint8_t* blk = reinterpret_cast<uint8_t*>(&s_blk[tid * 17]);
    for (uint32_t g = tid; g < ng; g += kThreads) {
      const uint32_t a = s.starts[g], b = s.starts[g + 1];
      uint64_t total = 0;
      uint32_t msg_len = 0;
      for (uint32_t j = a; j < b; ++j) msg_len += 68 + ndigits(cur_s[j]);
      uint32_t cv[8];
      zg::load_key(cv, zg::kNodeKeyW);
      uint32_t fill = 0, done = 0;  // bytes in the current block / bytes already compressed
      auto put = [&](uint32_t byte) {
        blk[fill++] = uint8_t(byte);
        if (fill == 64 && done + 64 < msg_len) {
          uint32_t m[16];
          const uint32_t* w = reinterpret_cast<const uint32_t*>(blk);
#pragma unroll
          for (int i = 0; i < 16; ++i) m[i] = w[i];
          zg::compress(cv, m, 0, 64, zg::KEYED_HASH | (done == 0 ? zg::CHUNK_START : 0u));
          done += 64;
          fill = 0;
        }
      };
      for (uint32_t j = a; j < b; ++j) {
        const uint64_t* hw = reinterpret_cast<const uint64_t*>(cur_h + 32 * size_t(j));
        for (int q = 0; q < 4; ++q) {
          const uint64_t v = hw[q];
          for (int d = 60; d >= 0; d -= 4) {
            const uint32_t nib = uint32_t(v >> d) & 15u;
            put(nib < 10 ? '0' + nib : 'a' + nib - 10);
          }
        }
        put(' ');
        put(':');
        put(' ');
        const uint64_t sz = cur_s[j];
        total += sz;
        uint64_t pw = 1;
        while (pw <= sz / 10) pw *= 10;
        for (; pw; pw /= 10) put('0' + uint32_t((sz / pw) % 10));
        put('\n');
      }
      for (uint32_t i = fill; i < 64; ++i) blk[i] = 0;
      uint32_t m[16];
      const uint32_t* w = reinterpret_cast<const uint32_t*>(blk);
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = w[i];
      zg::compress(cv, m, 0, fill, zg::KEYED_HASH | zg::CHUNK_END | zg::ROOT | (done == 0 ? zg::CHUNK_START : 0u));
      uint32_t* dst = reinterpret_cast<uint32_t*>(nxt_h + 32 * size_t(g));
      for (int k = 0; k < 8; ++k) dst[k] = cv[k];
      nxt_s[g] = total;
    }
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
  hipLaunchKernelGGL(k_merkle, dim3(n_jobs), dim3(kThreads), 0, stream, leaf_hashes, leaf_sizes, jobs, roots, scratch,
                     per_job / 256 * 256);
  return hipGetLastError();
}

}  // extern "C"
