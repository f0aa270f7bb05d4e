// Device-direct Xet pull (native GPU runtime, no Python): fetch a file's reconstruction terms through
// the cache -> P2P -> CDN waterfall into pinned staging, then decode (LZ4/BG4), BLAKE3-hash and
// Merkle-verify them on the GPU straight into a caller-provided HBM buffer.  Used by the pybind
// module (`_hip.DeviceXetPull`, zest_amd.direct / swarm_pull) and by the native per-GPU worker of
// `zest pull --gpus N` (csrc/gpurt/gpu_worker.cpp).
//
// Reference: the host equivalent is xet_bridge.zig:149-264 + parallel_download.zig:91-204 (fetch,
// then XorbReader.extractChunkRange on the CPU); here the CPU only moves compressed bytes.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "term_jobs.h"

namespace zest::gpurt {

struct DevicePullOptions {
  std::string repo;
  std::string revision = "main";
  std::string repo_type = "model";
  bool p2p = true;
  std::vector<std::string> peers;
  std::optional<std::string> tracker;
  bool dht = true;
  std::vector<std::string> dht_bootstrap;
  int device = 0;
  size_t staging_bytes = size_t(1) << 30;  // per pinned slot
  int slots = 0;                           // pinned staging slots (0: ZEST_DEVICE_SLOTS, default 3)
  int threads = 16;                        // fetch workers
  bool defer_device = false;  // construct the host side only; init_device() (or the first pull) does the rest
};

struct PullRequest {
  std::string xet_hash;  // Xet file hash (hex)
  uintptr_t dst = 0;     // device pointer
  uint64_t size = 0;     // file size (bytes)
};

struct PullFileStats {
  uint64_t bytes = 0, terms = 0, chunks = 0;
  double seconds = 0;          // whole call
  uint64_t fetched_bytes = 0;  // whole call (compressed bytes moved)
  std::vector<uint32_t> chunk_lens;  // uncompressed size of every chunk, in file order
};

// Called on the pipeline's releaser thread after a staging batch's kernels completed: file `file`
// (index into the request list) now holds its verified-or-not bytes [0, bytes) in HBM.  `attempt` is
// 0 for the first pass and 1 for the CDN repair pass of files whose Merkle root missed (which
// overwrites their bytes).  Keep it cheap: the next batch waits for it.
using PullProgressFn = std::function<void(size_t file, int attempt, uint64_t bytes)>;

class DeviceXetPull {
 public:
  explicit DeviceXetPull(const DevicePullOptions& opt);
  ~DeviceXetPull();
  DeviceXetPull(const DeviceXetPull&) = delete;
  DeviceXetPull& operator=(const DeviceXetPull&) = delete;
  // Pull several files through ONE pipeline (staging batches cross file boundaries; one Merkle
  // launch verifies all of them).  Throws zest::Error ("HashMismatch", "DownloadFailed", ...) when a
  // file cannot be verified after its CDN repair pass.
  std::vector<PullFileStats> pull_files(const std::vector<PullRequest>& files, const PullProgressFn& progress = {});
  // Term ranges of files (the term-sharded swarm pull, csrc/core/term_jobs.h): decoded into place at
  // each job's device address, chunk hashes / sizes into hashes[32 * i] / sizes[i] (device tables,
  // i = the job's chunk0 + chunk index).  Jobs must cover consecutive chunk indices.  No Merkle
  // check: the caller verifies each whole file, then settle(file, ok) publishes or drops the runs.
  std::vector<TermJobResult> pull_terms(const std::vector<TermJob>& jobs, uint8_t* hashes, uint64_t* sizes,
                                        bool repair = false);
  // Streaming form of pull_terms (the swarm pull's rounds): the jobs become one item of a continuous
  // pipeline that persists across items (no stream drain between them); returns a ticket at once.
  uint64_t submit_terms(const std::vector<TermJob>& jobs, uint8_t* hashes, uint64_t* sizes);
  struct ItemResult {
    std::string err;                     // empty: every term fetched and matched its plan
    std::vector<TermJobResult> results;  // per job (valid when err is empty)
    uintptr_t event = 0;                 // hipEvent_t completing with the item's kernels
  };
  // Blocks until the item's kernels are queued (not run) or it failed; once per ticket.
  ItemResult wait_item(uint64_t ticket);
  // The item's device decode error word (0 = clean); waits for its kernels.
  unsigned long long item_error(uint64_t ticket);
  // Wait for every submitted item (GPU included) and forget them and their events; `cancel` first
  // abandons the items still fetching (their remaining terms are skipped).
  void stream_reset(bool cancel = false);
  // Everything this pipeline queues from now on runs after the caller's hipEvent_t `event` completed.
  void order_after(uintptr_t event);
  size_t settle(const std::string& xet_hash, bool ok);
  std::vector<TermShape> term_shapes(const std::string& xet_hash);  // (ulen, chunks) per term
  std::vector<TermKey> term_keys(const std::string& xet_hash);      // (xorb hex, chunk range) per term
  // Which of the terms (xorb hex, chunk range) the local xorb cache holds (planner possession check).
  std::vector<uint8_t> cached_terms(const std::vector<std::string>& hexes, const std::vector<uint32_t>& starts,
                                    const std::vector<uint32_t>& ends);
  void reset_reconstructions();  // between pulls only
  std::string stats_json() const;
  size_t staging_bytes() const;
  // Device set-up (HIP streams, pinned + device staging) when the options deferred it.  Idempotent.
  void init_device();
  // A second pipeline (own streams and staging, `staging_bytes` per slot, 0 = this one's) over the
  // SAME host state: Xet session, caches, swarm, reconstructions and settle book.  The swarm pull
  // fetches round k + 1 on it while round k is agreed; settle() on either settles both's runs.
  std::unique_ptr<DeviceXetPull> sibling(size_t staging_bytes = 0, int slots = 0) const;
  // Wait for the write-behind cache queue (runs queued by fetches, and settle operations).
  void flush_cache_writes();
  std::string cache_writer_json() const;  // {"queued_bytes", "written_bytes", "dropped_bytes"}
  // ZEST_DEVICE_TIMING=1: the last pass's device timeline from timed HIP events around every
  // batch's H2D copy and kernels: {"batches", "window_ms", "h2d_busy_ms", "kernel_busy_ms",
  // "overlap_ms", "h2d_bytes", "h2d_GBps_busy"} ({} otherwise)
  std::string timeline_json() const;

  struct Shared;

 private:
  DeviceXetPull(const DevicePullOptions& opt, std::shared_ptr<Shared> shared);
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace zest::gpurt
