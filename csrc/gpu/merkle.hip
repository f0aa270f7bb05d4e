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

constexpr int kThreads = 256;
constexpr uint32_t kMsgBytes = 1024;  // 9 children * (64 + 3 + 20 + 1) = 792 < 1024

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
      s.flags[i] = word;
    }
    __syncthreads();
    if (tid == 0) {
      uint64_t p = 0;
      uint32_t g = 0;
      while (p < n) {
        s.starts[g++] = uint32_t(p);
        const uint64_t rem = n - p;
        uint64_t cut;
        if (rem <= 2) {
          cut = rem;
        } else {
          const uint64_t end = rem < 9 ? rem : 9;
          cut = end;
          for (uint64_t i = 2; i < end; ++i) {
            const uint64_t j = p + i;
            if ((s.flags[j >> 5] >> (j & 31)) & 1u) {
              cut = i + 1;
              break;
            }
          }
        }
        p += cut;
      }
      s.starts[g] = uint32_t(n);
      s_ngroups = g;
    }
    __syncthreads();
    const uint32_t ng = s_ngroups;
    uint8_t* nxt_h = into_a ? s.hash_a : s.hash_b;
    uint64_t* nxt_s = into_a ? s.size_a : s.size_b;
    uint8_t* msg = s.msg + size_t(tid) * kMsgBytes;
    for (uint32_t g = tid; g < ng; g += kThreads) {
      const uint32_t a = s.starts[g], b = s.starts[g + 1];
      uint32_t pos = 0;
      uint64_t total = 0;
      for (uint32_t j = a; j < b; ++j) {
        pos = put_line(msg, pos, cur_h + 32 * size_t(j), cur_s[j]);
        total += cur_s[j];
      }
      uint32_t cv[8];
      zg::hash_chunk(msg, pos, 0, zg::kNodeKeyW, zg::KEYED_HASH, true, cv);
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
