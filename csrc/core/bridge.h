// XetBridge: the cache -> P2P -> CDN waterfall for one reconstruction term, plus fetch stats.
//
// Reference: src/xet_bridge.zig:1-307 — authenticate via xet-read-token (:76-130),
// getReconstruction (:133-142), fetchXorbForTerm (:149-218) using the FetchInfo that covers the
// term (:221-228), caching every CDN entry full/partial for seeding, returning local (rebased)
// chunk indices; printStats strings (:267-281) are preserved verbatim.  Stats are atomics here
// (the reference races on them from concurrent tasks, SURVEY §5.2 a).
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <optional>
#include <ostream>
#include <functional>
#include <string>

#include "config.h"
#include "hub.h"
#include "storage.h"
#include "swarm.h"

namespace zest {

struct FetchStats {
  std::atomic<uint64_t> xorbs_from_cache{0}, xorbs_from_peer{0}, xorbs_from_cdn{0};
  std::atomic<uint64_t> bytes_from_cache{0}, bytes_from_peer{0}, bytes_from_cdn{0};
  std::atomic<uint64_t> verify_failures{0}, refetches{0};
};

// Resumed: restored from a .zest-resume sidecar (bytes written by an earlier, interrupted run).
enum class Source { Cache, Peer, Cdn, Resumed };

struct FetchOptions {
  bool allow_p2p = true;
  bool allow_cache = true;
  // CDN refetch repairing a copy that failed verification: the CDN run replaces whatever the
  // cache holds under its name (put_run normally keeps an existing longer run).
  bool repair = false;
  // With a write-behind writer and a sink: the cache copy of a run received into sink memory is
  // made by the writer's copy threads instead of this thread; on_copied() runs once they have it
  // (XorbFetchResult::copy_deferred says whether it will run).  The caller keeps the sink memory.
  std::function<void()> on_copied;
};

struct XorbFetchResult {
  Bytes data;
  uint32_t local_start = 0, local_end = 0;  // chunk indices inside the fetched run
  Source source = Source::Cdn;
  std::string peer;
  // Cache bookkeeping for verification: Cache -> the run the hit came from (evicted when the file
  // fails verification); Peer -> the run quarantined with put_pending (`pending` = its quarantine
  // file, unique to this fetch), published by XetBridge::settle once the file hash checked out.
  uint32_t run_offset = 0;
  std::string pending;
  // With a sink: the run was written to sink memory instead of `data`.
  uint8_t* ext = nullptr;
  size_t ext_len = 0;
  bool copy_deferred = false;  // FetchOptions::on_copied will run (a writer copy thread owns the cache copy)
  const uint8_t* bytes() const { return ext ? ext : data.data(); }
  size_t size() const { return ext ? ext_len : data.size(); }
};

class XetBridge {
 public:
  XetBridge(const Config& cfg, storage::XorbCache* cache, SwarmDownloader* swarm)
      : cfg_(cfg), cache_(cache), swarm_(swarm) {}
  void authenticate(const std::string& repo_id, const std::string& repo_type, const std::string& revision);
  void set_cas(const std::string& cas_url, const std::string& token);
  bool authenticated() const { return cas_ != nullptr; }
  cas::Reconstruction get_reconstruction(const std::string& file_hash_hex) const;
  // `sink` (optional) supplies destination memory for the fetched run (e.g. a pinned staging
  // region); when it returns nullptr the run lands in XorbFetchResult::data as usual.
  XorbFetchResult fetch_term(const cas::Term& term, const cas::Reconstruction& recon, const FetchOptions& opt = {},
                             const bt::PayloadSink& sink = {});
  // After the file a term belongs to was verified (ok) or failed (!ok): publish or drop a peer
  // run quarantined by fetch_term; on failure also evict the cached run a cache hit came from, so
  // the repair refetch cannot read the same bad bytes again.
  void settle(const std::string& xorb_hex, const XorbFetchResult& r, bool ok);
  void settle(const std::string& xorb_hex, Source src, uint32_t run_offset, const std::string& pending, bool ok);
  FetchStats& stats() { return stats_; }
  void print_stats(std::ostream& w) const;
  std::string stats_json() const;
  SwarmDownloader* swarm() { return swarm_; }
  // Route cache writes (CDN runs, quarantined peer runs, and the settle operations behind them)
  // through a write-behind queue instead of the fetch thread (device pulls; see storage::CacheWriter).
  void set_writer(storage::CacheWriter* w) { writer_ = w; }
  storage::CacheWriter* writer() const { return writer_; }
  // Runs the write-behind queue had no room for (dropped instead of stalling the fetch): recorded
  // here, and fill_deferred() fetches them again from the CDN -- the trusted origin, so a dropped
  // quarantined peer run is replaced by a verified one -- and writes them into the cache once the
  // pull's hot path is over.  Seed-while-downloading then misses nothing (the
  // reference always caches after a fetch, swarm.zig:416-420).  Returns the runs written.
  size_t fill_deferred();
  size_t deferred_count() const;

 private:
  void defer(const std::string& hex, const cas::FetchInfo& fi, bool repair);
  const Config& cfg_;
  storage::XorbCache* cache_;
  SwarmDownloader* swarm_;
  storage::CacheWriter* writer_ = nullptr;
  std::unique_ptr<cas::CasClient> cas_;
  FetchStats stats_;
  struct Deferred {
    std::string hex;
    cas::FetchInfo fi;
    bool repair = false;
  };
  mutable std::mutex deferred_mu_;
  std::vector<Deferred> deferred_;
};

}  // namespace zest
