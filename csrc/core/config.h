// Runtime configuration (environment + defaults), shared by the CLI, servers and Python.
//
// Reference: src/config.zig:1-183 — defaults hub https://huggingface.co, revision main, DHT/listen
// port 6881, HTTP 9847, max_peers 50, chunk target 65536, 16 concurrent downloads (:6-13);
// env HOME, HF_HOME, ZEST_CACHE_DIR, HF_TOKEN (else ~/.cache/huggingface/token), ZEST_HTTP_PORT,
// ZEST_MAX_PEERS (:37-84, :136-158).
// Deliberate deviation: HF cache follows real huggingface_hub semantics
// (HF_HUB_CACHE > $HF_HOME/hub > ~/.cache/huggingface/hub) instead of using HF_HOME as the hub dir,
// and the hub endpoint honours HF_ENDPOINT (used by the offline fake hub in tests).
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "sha1.h"

namespace zest {

constexpr const char* kVersion = "0.4.2";
constexpr const char* kDefaultHub = "https://huggingface.co";
constexpr const char* kDefaultRevision = "main";
constexpr uint16_t kDefaultDhtPort = 6881;
constexpr uint16_t kDefaultListenPort = 6881;
constexpr uint16_t kDefaultHttpPort = 9847;
constexpr uint32_t kDefaultMaxPeers = 50;
constexpr uint32_t kDefaultChunkTarget = 65536;
constexpr uint32_t kDefaultConcurrency = 16;
// Public BitTorrent DHT routers (reference: config.zig:14-18 and dht.zig:32-36 list them but never
// bootstrap from them; router.utorrent.com added).
constexpr const char* kDefaultDhtRouters[] = {"router.bittorrent.com:6881", "dht.transmissionbt.com:6881",
                                              "router.utorrent.com:6881"};

struct Config {
  std::string home;
  std::string hub_url;
  std::string hf_cache_dir;    // .../hub
  std::string cache_dir;       // ~/.cache/zest
  std::string xorb_cache_dir;  // cache_dir/xorbs
  std::string chunk_cache_dir; // cache_dir/chunks
  std::string pid_file;
  std::optional<std::string> hf_token;
  peer_id::PeerId peer_id{};
  uint16_t dht_port = kDefaultDhtPort;
  uint16_t listen_port = kDefaultListenPort;
  uint16_t http_port = kDefaultHttpPort;
  uint32_t max_peers = kDefaultMaxPeers;
  uint32_t max_inbound = 512;      // ZEST_MAX_INBOUND: concurrent peer connections the seeding server serves
  uint32_t peer_connections = 16;  // ZEST_PEER_CONNECTIONS: parallel connections per peer (= default concurrency)
  uint32_t chunk_target = kDefaultChunkTarget;
  uint32_t concurrency = kDefaultConcurrency;
  int connect_timeout_ms = 5000;
  int io_timeout_ms = 30000;
  int discovery_ttl_s = 30;
  // DHT bootstrap routers used when no --dht-bootstrap is given; ZEST_DHT_BOOTSTRAP="h:p,..."
  // replaces them ("none" = no default bootstrap).
  std::vector<std::string> dht_routers;
  // MI355X extensions
  int gpus = 0;             // ZEST_GPUS (0 = CPU verify path)
  double hbm_cache_gb = 0;  // ZEST_HBM_CACHE_GB
  bool trace = false;       // ZEST_TRACE
  std::string fault;        // ZEST_FAULT ("drop:p,corrupt:p,delay:ms")
  bool cache_writes = true; // ZEST_CACHE_WRITES=0: do not keep fetched runs in the xorb cache
  double cache_max_gb = 0;  // ZEST_CACHE_MAX_GB: trim the xorb cache (least recently used runs) to this size; 0 = unbounded

  static Config from_env();
  std::string repo_dir(const std::string& repo_id) const;  // models--org--name
  std::string snapshot_dir(const std::string& repo_id, const std::string& commit) const;
  std::string xorb_cache_path(const std::string& key) const;   // xorbs/{key[0..2]}/{key}
  std::string chunk_cache_path(const std::string& key) const;  // chunks/{key[0..2]}/{key}
  std::string to_json() const;
};

std::string repo_folder_name(const std::string& repo_id, const std::string& type = "model");

}  // namespace zest
