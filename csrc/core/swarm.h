// Swarm orchestration: peer discovery (DHT + tracker, TTL-cached), direct peers, pooled BEP XET
// fetches, announce/seed bookkeeping and download statistics.
//
// Reference: src/swarm.zig:150-486 — SwarmDownloader with DHT, tracker, PeerPool, direct peers,
// discovered-peer cache with a 30 s TTL (:182-254), discoverPeers (:320-355), sequential
// tryBtPeerDownload over direct then cached peers (:363-394), tryPooledChunkDownload (:398-437),
// announceToSwarm (:458-470), printStats (:472-485).  Differences: counters are atomics (the
// reference mutates stats from concurrent tasks without a lock, SURVEY §5.2 a/b), the cached peer
// list is copied under the lock before iteration (§5.2 c), peers that time out or serve corrupt
// data are scored down and skipped, and terms are striped over every known peer: each request goes
// to the candidate with the fewest requests in flight (the reference tries peers in fixed order,
// first success wins, so one seeder serves everything, swarm.zig:371-394).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <ostream>
#include <string>
#include <thread>
#include <vector>

#include "bt_peer.h"
#include "config.h"
#include "dht.h"
#include "storage.h"
#include "xet_hash.h"

namespace zest {

struct DownloadStats {
  std::atomic<uint64_t> total_xorbs{0}, cached_xorbs{0}, peer_xorbs{0}, cdn_xorbs{0};
  std::atomic<uint64_t> total_bytes{0}, peer_bytes{0}, peers_connected{0}, dht_lookups{0}, tracker_announces{0};
  std::atomic<uint64_t> peer_failures{0}, peers_banned{0};
};

class SwarmDownloader {
 public:
  SwarmDownloader(const Config& cfg, std::optional<std::string> tracker_url, bool enable_p2p,
                  bool enable_dht = true, std::vector<net::Addr> dht_bootstrap = {});
  ~SwarmDownloader();
  void add_direct_peer(const net::Addr& a);
  bool p2p_enabled() const { return enabled_; }
  // Fetch chunks [start, end) of xorb `hash` from any peer; nullopt if no peer could serve it.
  std::optional<bt::ChunkResult> try_peers(const xet::Hash& hash, uint32_t start, uint32_t end,
                                           const bt::PayloadSink& sink = {});
  std::vector<net::Addr> discover(const Sha1Digest& info_hash);
  void announce(const std::vector<xet::Hash>& xorbs);
  // A peer served bytes that failed verification: ban it for the rest of the session.
  void report_bad_peer(const std::string& addr);
  DownloadStats& stats() { return stats_; }
  void print_stats(std::ostream& os) const;
  // Bytes each peer served this session ("addr" -> bytes), for stats / striping checks.
  std::map<std::string, uint64_t> peer_bytes() const;
  dht::Dht* dht() { return dht_.get(); }
  // The background bootstrap from the default routers finished (or there was none to run).
  bool bootstrap_done() const { return boot_done_ || !boot_thread_.joinable(); }

 private:
  const Config& cfg_;
  bool enabled_;
  std::optional<std::string> tracker_;
  std::unique_ptr<dht::Dht> dht_;
  std::unique_ptr<bt::PeerPool> pool_;
  std::vector<net::Addr> direct_;
  mutable std::mutex mu_;
  struct Cached {
    std::vector<net::Addr> peers;
    std::chrono::steady_clock::time_point at;
  };
  std::map<std::string, Cached> discovered_;
  std::map<std::string, int> score_;  // addr -> failures
  std::set<std::string> served_by_;   // distinct peers that served data ("Peers connected")
  std::vector<net::Addr> known_;      // peers that served or were discovered, tried before per-xorb discovery
  std::set<std::string> known_keys_;
  // Per-peer load for striping: requests in flight, bytes served, range hits and misses.
  struct PeerLoad {
    int inflight = 0;
    uint64_t bytes = 0;
    uint32_t hits = 0, misses = 0;
    std::chrono::steady_clock::time_point window{};  // start of the current miss-count window
  };
  // Miss counts are forgotten every `miss_decay_` (ZEST_PEER_MISS_DECAY_S, default 30 s = the
  // discovery TTL): a peer that missed early -- it was pulling the same model at the same time --
  // is tried again once it may have the xorbs (the reference re-discovers on a TTL, swarm.zig:324-330).
  std::chrono::steady_clock::duration miss_decay_ = std::chrono::seconds(30);
  std::map<std::string, PeerLoad> load_;
  void remember(const net::Addr& a);  // caller holds mu_
  std::mutex disc_mu_;
  DownloadStats stats_;
  // DHT re-announce of xorbs fetched from peers: queued and drained by an owned worker thread
  // (never a detached thread holding `this`).
  void announce_worker();
  void bootstrap_default();
  std::thread boot_thread_;
  std::atomic<bool> boot_done_{false};
  std::mutex aq_mu_;
  std::condition_variable aq_cv_;
  std::vector<Sha1Digest> announce_q_;
  bool aq_stop_ = false;
  std::thread aq_thread_;
};

}  // namespace zest
