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
#include <memory>
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
  std::vector<uint32_t> chunk_lens;  // uncompressed chunk sizes in file order (memory targets)
};

class ParallelDownloader {
 public:
  ParallelDownloader(XetBridge& bridge, int concurrency)
      : bridge_(bridge), concurrency_(concurrency), free_(size_t(std::max(1, concurrency))) {
    for (size_t i = 0; i < free_; ++i) bufs_.push_back(std::make_unique<RunBuffer>());
  }
  // Optional hook: called with every verified-in-order byte range (file offset, bytes) after the
  // file hash check, e.g. to stage the file into device memory.
  using RangeHook = std::function<void(uint64_t, const uint8_t*, size_t)>;
  // Thread-safe: several files may be reconstructed at once (pull.cpp runs a few Xet files
  // concurrently).  Their workers share one gate of `concurrency` term slots, so at most that many
  // terms are in flight in total, and one file's tail (its last few terms) is filled with the next
  // file's terms instead of idle workers.
  // `on_term(bytes, source)` (optional) is called as each term lands in the file.
  FileResult reconstruct_to_file(const std::string& file_hash_hex, const std::string& out_path, bool verify = true,
                                 const std::function<void(uint64_t, Source)>& on_term = {});
  // Same waterfall + verification into caller memory (`cap` >= the file size); no file, no resume
  // sidecar.  FileResult::chunk_lens carries the chunk boundaries (e.g. for a swarm receiver).
  FileResult reconstruct_to_memory(const std::string& file_hash_hex, uint8_t* dst, uint64_t cap, bool verify = true,
                                   const std::function<void(uint64_t, Source)>& on_term = {});

 private:
  FileResult reconstruct(const std::string& hex, const std::string& out_path, uint8_t* mem, uint64_t mem_cap,
                         bool verify, const std::function<void(uint64_t, Source)>& on_term);
  // One receive buffer per term slot, kept across terms and files: a fetched run (up to a 64 MiB
  // xorb) lands in memory whose pages were faulted in once, instead of a fresh mmap'd allocation
  // per term whose every page faults and is zeroed on first touch.
  struct RunBuffer {
    std::unique_ptr<uint8_t[]> p;
    size_t cap = 0;
    uint8_t* get(size_t n) {
      if (n > cap) {
        p.reset(new uint8_t[n]);
        cap = n;
      }
      return p.get();
    }
  };
  RunBuffer* acquire_slot();
  void release_slot(RunBuffer* b);

  XetBridge& bridge_;
  int concurrency_;
  std::mutex gate_mu_;
  std::condition_variable gate_cv_;
  size_t free_;
  std::vector<std::unique_ptr<RunBuffer>> bufs_;  // the free slots' buffers
};

}  // namespace zest
