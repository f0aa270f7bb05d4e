// `zest pull`: list repo files, resolve the commit, authenticate with Xet CAS, reconstruct every
// Xet file through the cache -> P2P -> CDN waterfall, download regular files, write the HF cache
// layout (snapshots/{commit}/..., refs/{revision}) and print the reference's stats block.
//
// Reference: src/main.zig:83-305 (cmdPull) with its fallbacks: parallel -> sequential bridge ->
// opaque CDN download (main.zig:233-256); a file is "(cached)" only if it exists — here cached
// files must also match their size (a crashed run leaves `.incomplete`, never a final name).
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <optional>
#include <ostream>
#include <string>
#include <vector>

#include "config.h"
#include "net.h"

namespace zest {

// Live progress of one pull (read by the REST API's /v1/pull SSE stream while the pull runs).
struct PullProgress {
  struct File {
    std::string path;
    uint64_t size = 0;
    std::atomic<uint64_t> done{0};
    std::atomic<int> state{0};  // 0 queued, 1 running, 2 done, 3 failed, 4 cached
  };
  std::atomic<bool> listed{false};
  std::atomic<uint64_t> bytes{0}, total{0};
  std::atomic<uint64_t> from_peer{0}, from_cdn{0}, from_cache{0};
  std::atomic<int> last_source{0};  // 0 none, 1 cache, 2 peer, 3 cdn (source of the latest term)
  std::atomic<uint32_t> peers{0};
  std::mutex mu;                     // guards `files` growth (set once after listing)
  std::vector<std::unique_ptr<File>> files;
  void add(size_t file, uint64_t n, int source);
  static const char* source_name(int s);
};

struct PullOptions {
  std::string repo_id;
  std::string revision = "main";
  std::string repo_type = "model";
  std::optional<std::string> tracker;
  std::vector<std::string> peers;           // --peer ip:port (repeatable)
  std::vector<std::string> dht_bootstrap;   // --dht-bootstrap host:port
  bool p2p = true;
  bool dht = true;
  bool verify = true;
  int concurrency = 0;                      // 0 = cfg.concurrency
  bool autostart_server = true;
  std::vector<std::string> include;         // optional path filters (suffix match)
  std::shared_ptr<PullProgress> progress;   // optional live progress sink
};

struct PullSummary {
  std::string snapshot_dir;
  std::string commit;
  uint64_t bytes = 0;
  size_t files = 0, xet_files = 0, cached_files = 0;
  uint64_t bytes_from_peer = 0, bytes_from_cdn = 0, bytes_from_cache = 0;
  double seconds = 0;
  std::string stats_json;
  std::string files_json;  // [{"path","size","xet_hash"|null,"ok"}] for every listed file
  size_t failed_files = 0;
};

PullSummary run_pull(Config& cfg, const PullOptions& opt, std::ostream& out, std::ostream& err);

// Background server helpers shared by the CLI and the HTTP API.
bool server_healthy(uint16_t http_port, int timeout_ms = 1000);
bool spawn_background_server(const std::string& self_exe, uint16_t http_port);

}  // namespace zest
