// Term-range fetch jobs: the unit of work of the term-sharded intra-node swarm pull
// (zest_amd.parallel.swarm_pull).  A job is a contiguous range of one Xet file's reconstruction
// terms, fetched through the cache -> P2P -> CDN waterfall and decoded + chunk-hashed straight into
// the caller's memory at the range's output offset.  Unlike a whole-file pull, nothing here can
// check a Merkle root (a term range is part of a file): the caller collects every chunk hash of a
// file -- its own and the ones it re-derives from bytes received from peer ranks -- checks the file
// hash, then settles the file's runs (publish quarantined peer runs, or drop and evict them before a
// CDN repair fetch).
//
// Reference: parallel_download.zig:91-204 fetches whole files' terms with 16 concurrent tasks and
// never verifies; xet_bridge.zig:149-218 is the per-term waterfall reused here through XetBridge.
#pragma once

#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "bridge.h"

namespace zest {

struct TermJob {
  std::string xet_hash;  // file
  uint32_t t0 = 0, t1 = 0;  // term range [t0, t1) of the file's reconstruction
  uintptr_t dst = 0;        // address of term t0's first output byte (host or device memory)
  uint64_t chunk0 = 0;      // index of term t0's first chunk in the caller's hash table
};

struct TermJobResult {
  std::vector<uint32_t> chunk_lens;  // uncompressed size of every chunk of the range, in order
  uint64_t fetched = 0;              // bytes moved for the range (compressed runs)
  uint64_t from_peer = 0, from_cdn = 0, from_cache = 0;  // unpacked bytes by source
};

// (unpacked_length, chunk count) of every term of a file, in reconstruction order.
struct TermShape {
  uint64_t ulen = 0;
  uint32_t nchunks = 0;
};

// (xorb hex, chunk range start, end) of every term of a file, in reconstruction order.
struct TermKey {
  std::string hex;
  uint32_t start = 0, end = 0;
};

// Thread-safe reconstruction cache: the planner asks once per file, the fetch jobs reuse it.
class ReconCache {
 public:
  explicit ReconCache(XetBridge& bridge) : bridge_(bridge) {}
  const cas::Reconstruction& get(const std::string& hex);
  std::vector<TermShape> shapes(const std::string& hex);
  std::vector<TermKey> keys(const std::string& hex);
  // Forget every reconstruction (the next pull asks the CAS again: presigned URLs expire).  Only
  // between pulls: references handed out by get() die with it.
  void clear();

 private:
  XetBridge& bridge_;
  std::mutex mu_;
  std::map<std::string, cas::Reconstruction> recs_;
};

// Cache runs behind fetched terms, held per file until the file's verdict is known.
class SettleBook {
 public:
  void add(const std::string& file_hex, const std::string& xorb_hex, Source src, uint32_t run_offset,
           const std::string& pending);
  // Publish (ok) or drop / evict (!ok) every run recorded for the file; returns how many.
  size_t settle(XetBridge& bridge, const std::string& file_hex, bool ok);
  size_t settle_all(XetBridge& bridge, bool ok);
  // Drop the quarantined peer runs (file hex, pending path) a failed call recorded; returns how many.
  size_t discard(XetBridge& bridge, const std::vector<std::pair<std::string, std::string>>& runs);

 private:
  struct Run {
    std::string xorb_hex;
    Source src;
    uint32_t run_offset;
    std::string pending;
  };
  std::mutex mu_;
  std::map<std::string, std::vector<Run>> runs_;
};

// Possession check of the swarm planner: 1 per term (xorb hex, chunk range [start, end)) that the
// local xorb cache covers, 0 otherwise; `threads` workers check terms concurrently.
std::vector<uint8_t> cached_terms(const storage::XorbCache& cache, const std::vector<std::string>& hexes,
                                  const std::vector<uint32_t>& starts, const std::vector<uint32_t>& ends, int threads);

// Host twin of DeviceXetPull::pull_terms: `threads` workers fetch the jobs' terms, decode and hash
// every chunk on the CPU, write the bytes at job.dst (host memory) and the keyed-BLAKE3 chunk hashes
// at hashes + 32 * chunk index.  A term whose copy does not decode is refetched from the CDN once
// (its peer/cache run rejected); `repair` fetches everything from the CDN, replacing cached runs.
// Throws on a term that fails from every source.
std::vector<TermJobResult> fetch_terms_host(XetBridge& bridge, ReconCache& recs, SettleBook& book,
                                            const std::vector<TermJob>& jobs, uint8_t* hashes, int threads,
                                            bool repair);

// [lo, hi) byte ranges covering the runs (at[i], len[i]) of a staging slot, in address order, with
// neighbours whose gap is at most max_gap merged (one copy command instead of two); empty runs are
// skipped.  The device pull copies only these to the GPU, not the holes between reserved regions.
std::vector<std::pair<uint64_t, uint64_t>> copy_ranges(const std::vector<uint64_t>& at,
                                                       const std::vector<uint64_t>& len, uint64_t max_gap);

}  // namespace zest
