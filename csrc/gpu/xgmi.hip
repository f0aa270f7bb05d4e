// K8: pull-mode peer gather over xGMI for the `xgmi` exchange (zest_amd/engine.py).
//
// Every rank maps its peers' HBM arenas (HIP IPC) and, per round, copies each peer's freshly
// verified region into its own arena.  One launch covers every peer: block b serves segment
// b % nseg, so all peers — hence all 7 point-to-point xGMI links of an MI355X — are read at once,
// instead of one DMA copy per peer queued on a handful of streams.  Loads are 16 B per lane,
// 8 in flight per lane before the stores (remote reads have microsecond latency), stores are
// non-temporal: the received bytes are hashed once and never re-read from L2.
//
// No reference equivalent: the reference moves xorbs between hosts over BT TCP
// (src/bt_peer.zig); this is the intra-node replacement (SURVEY §5.8 "direct P2P all-to-all").
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "zgpu.h"

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kUnroll = 8;

__global__ __launch_bounds__(kThreads) void k_peer_gather(ZgPeerSegs s, uint32_t blocks_per_seg) {
  const uint32_t seg = blockIdx.x % uint32_t(s.nseg);
  const uint32_t sb = blockIdx.x / uint32_t(s.nseg);
  const uint8_t* src = reinterpret_cast<const uint8_t*>(s.src[seg]);
  uint8_t* dst = reinterpret_cast<uint8_t*>(s.dst[seg]);
  const uint64_t n = s.n[seg];
  // src and dst are congruent mod 16 (host-checked): byte head up to 16 B alignment, vector body,
  // byte tail.
  uint64_t head = (16 - (s.dst[seg] & 15)) & 15;
  if (head > n) head = n;
  const uint64_t nv = (n - head) >> 4;
  const uint64_t tail0 = head + (nv << 4);
  if (sb == 0 && threadIdx.x < 16) {
    if (threadIdx.x < head) dst[threadIdx.x] = src[threadIdx.x];
    if (tail0 + threadIdx.x < n) dst[tail0 + threadIdx.x] = src[tail0 + threadIdx.x];
  }
  const v4u* s4 = reinterpret_cast<const v4u*>(src + head);
  v4u* d4 = reinterpret_cast<v4u*>(dst + head);
  const uint64_t stride = uint64_t(blocks_per_seg) * kThreads * kUnroll;
  for (uint64_t base = uint64_t(sb) * kThreads * kUnroll + threadIdx.x; base < nv; base += stride) {
    v4u v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t i = base + uint64_t(u) * kThreads;
      if (i < nv) v[u] = __builtin_nontemporal_load(s4 + i);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t i = base + uint64_t(u) * kThreads;
      if (i < nv) __builtin_nontemporal_store(v[u], d4 + i);
    }
  }
}

}  // namespace

extern "C" hipError_t zg_peer_gather(const ZgPeerSegs* segs, hipStream_t stream) {
  if (segs->nseg <= 0) return hipSuccess;
  if (segs->nseg > kZgMaxPeerSegs) return hipErrorInvalidValue;
  uint64_t max_n = 0;
  for (int i = 0; i < segs->nseg; ++i) {
    if ((segs->src[i] & 15) != (segs->dst[i] & 15)) return hipErrorInvalidValue;
    if (segs->n[i] > max_n) max_n = segs->n[i];
  }
  if (max_n == 0) return hipSuccess;
  // At most ~2 blocks per CU (512 over 256 CUs; ZG_PEER_GATHER_BLOCKS overrides), at least one per
  // segment.  The gather runs next to the round's decode and hash kernels, and the decoder is
  // occupancy-bound (profiles/lz4_records_r3.md): a grid of 8 blocks per CU would take every wave
  // slot for the whole transfer.  512 blocks keep 512 x 256 lanes x 128 B = 16 MiB of remote reads
  // in flight, far above the bandwidth-delay product of 7 links (~350 GB/s x a few us).
  static const uint64_t total = [] {
    const char* v = getenv("ZG_PEER_GATHER_BLOCKS");
    const long b = v ? atol(v) : 512;
    return uint64_t(b < 1 ? 1 : b > 8192 ? 8192 : b);
  }();
  const uint64_t per_block = uint64_t(kThreads) * kUnroll * 16;
  uint64_t bps = (max_n + per_block - 1) / per_block;
  const uint64_t cap = total / uint64_t(segs->nseg);
  if (bps > cap) bps = cap;
  if (bps < 1) bps = 1;
  hipLaunchKernelGGL(k_peer_gather, dim3(uint32_t(bps) * uint32_t(segs->nseg)), dim3(kThreads), 0, stream, *segs,
                     uint32_t(bps));
  return hipGetLastError();
}
