// ParallelDownloader: reconstruct one Xet file from its terms with N concurrent fetch workers,
// verify it end-to-end, and resume after a crash.
//
// Reference: src/parallel_download.zig:1-230 — batches of min(terms, 16*8) concurrent
// fetchXorbForTerm + extractChunkRange tasks, a barrier per batch, ordered writes, first error
// aborts (:91-204).  Here: a sliding window (workers pull the next term as soon as they finish;
// each term's output offset is known, so results are pwrite()n directly — no barrier, bounded
// memory), every chunk is hashed while extracting and the Merkle file hash is compared with the
// file's Xet hash; terms that came from peers are re-fetched from the CDN on mismatch (and the
// peers banned).  Output goes to `<path>.incomplete` with a `<path>.zest-resume` sidecar
// recording completed terms + their chunk hashes (the reference leaves truncated files that later
// count as cached), then is renamed into place.
#pragma once

#include <cstdint>
#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "bridge.h"

namespace zest {

struct FileResult {
  uint64_t bytes = 0;
  size_t terms = 0;
  size_t resumed_terms = 0;
  bool verified = false;
  double seconds = 0;
};

class ParallelDownloader {
 public:
  ParallelDownloader(XetBridge& bridge, int concurrency)
      : bridge_(bridge), concurrency_(concurrency), free_(size_t(std::max(1, concurrency))) {}
  // Optional hook: called with every verified-in-order byte range (file offset, bytes) after the
  // file hash check, e.g. to stage the file into device memory.
  using RangeHook = std::function<void(uint64_t, const uint8_t*, size_t)>;
  // Thread-safe: several files may be reconstructed at once (pull.cpp runs a few Xet files
  // concurrently).  Their workers share one gate of `concurrency` term slots, so at most that many
  // terms are in flight in total, and one file's tail (its last few terms) is filled with the next
  // file's terms instead of idle workers.
  FileResult reconstruct_to_file(const std::string& file_hash_hex, const std::string& out_path, bool verify = true);

 private:
  void acquire_slot();
  void release_slot();

  XetBridge& bridge_;
  int concurrency_;
  std::mutex gate_mu_;
  std::condition_variable gate_cv_;
  size_t free_;
};

}  // namespace zest
