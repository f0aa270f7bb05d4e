// Kademlia DHT (BEP 5) over UDP: routing table, KRPC codec, a query server and iterative
// get_peers / announce_peer lookups.
//
// Reference: src/dht.zig:1-671 — XOR metric (:41-54), 160 k-buckets of K=8 (:16, :120-128),
// KRPC builders with pre-sorted keys (:171-239), compact nodes 26 B / peers 6 B (:251-331).
// The reference DHT is inert (bootstrap() is never called, get_peers is a single
// round with no timeout, announce uses a fake token "zest").  This one bootstraps, runs an
// iterative α=3 lookup with deadlines, answers queries itself (so local zest nodes form a DHT),
// issues/validates real tokens and remembers announced peers.
#pragma once

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "net.h"
#include "sha1.h"

namespace zest::dht {

constexpr int K = 8;
constexpr int ALPHA = 3;
using NodeId = std::array<uint8_t, 20>;

NodeId xor_distance(const NodeId& a, const NodeId& b);
bool closer(const NodeId& target, const NodeId& a, const NodeId& b);  // a strictly closer than b
int bucket_index(const NodeId& own, const NodeId& other);             // 0..159, -1 if equal
NodeId random_id();

struct NodeInfo {
  NodeId id{};
  net::Addr addr;
};

class RoutingTable {
 public:
  explicit RoutingTable(const NodeId& own) : own_(own), buckets_(160) {}
  // Insert or refresh; a full bucket keeps its existing nodes (drops the newcomer).
  bool insert(const NodeInfo& n);
  void remove(const NodeId& id);
  std::vector<NodeInfo> closest(const NodeId& target, size_t k = K) const;
  size_t size() const;
  const NodeId& own() const { return own_; }

 private:
  NodeId own_;
  std::vector<std::vector<NodeInfo>> buckets_;
  mutable std::mutex mu_;
};

// KRPC messages (bencoded, keys sorted).
std::string build_ping(std::string_view tid, const NodeId& own);
std::string build_find_node(std::string_view tid, const NodeId& own, const NodeId& target);
std::string build_get_peers(std::string_view tid, const NodeId& own, const Sha1Digest& info_hash);
std::string build_announce_peer(std::string_view tid, const NodeId& own, const Sha1Digest& info_hash,
                                uint16_t port, std::string_view token, bool implied_port = false);
std::vector<NodeInfo> parse_compact_nodes(std::string_view data);
std::string encode_compact_node(const NodeInfo& n);

struct DhtStats {
  uint64_t queries_sent = 0, responses = 0, queries_answered = 0, timeouts = 0, lookups = 0;
};

class Dht {
 public:
  // Bind UDP on `port` (0 = ephemeral).  A bind failure leaves a socket-less DHT (like the
  // reference, dht.zig:350-360) that answers every lookup with no peers.
  Dht(uint16_t port, NodeId own = random_id());
  ~Dht();
  void start();
  void stop();
  bool has_socket() const { return sock_.valid(); }
  uint16_t port() const { return port_; }
  const NodeId& id() const { return table_.own(); }
  RoutingTable& table() { return table_; }

  // Ping + find_node(own id) against the given nodes to populate the table.
  size_t bootstrap(const std::vector<net::Addr>& nodes, int timeout_ms = 2000);
  // Iterative lookup; returns peers for info_hash (and caches tokens for announce).
  std::vector<net::Addr> get_peers(const Sha1Digest& info_hash, int timeout_ms = 3000);
  // Announce to the K closest nodes that handed us tokens (runs a lookup if needed).
  size_t announce_peer(const Sha1Digest& info_hash, uint16_t port, int timeout_ms = 3000);
  bool ping(const net::Addr& a, int timeout_ms = 1000);
  DhtStats stats() const;
  // Locally stored peers (from announces we received).
  std::vector<net::Addr> stored_peers(const Sha1Digest& info_hash) const;

 private:
  struct Pending {
    bool done = false;
    std::string reply;
    net::Addr from;
  };
  bool rpc(const net::Addr& to, const std::string& msg, const std::string& tid, int timeout_ms, std::string& reply);
  std::string next_tid();
  void recv_loop();
  void handle_query(const std::string& pkt, const net::Addr& from);
  std::string token_for(const net::Addr& a) const;

  net::Socket sock_;
  uint16_t port_ = 0;
  RoutingTable table_;
  std::thread thr_;
  std::atomic<bool> stop_{false};
  std::atomic<uint32_t> tid_{0};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, Pending> pending_;
  std::map<std::string, std::vector<std::pair<net::Addr, std::string>>> tokens_;  // ih -> (node, token)
  std::map<std::string, std::vector<net::Addr>> store_;                              // ih -> peers
  std::string secret_;
  DhtStats stats_;
};

}  // namespace zest::dht
