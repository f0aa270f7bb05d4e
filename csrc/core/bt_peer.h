// Client side of one BitTorrent peer connection speaking BEP 10 + BEP XET, with request
// pipelining, plus the connection pool.
//
// Reference: src/bt_peer.zig:1-346 (connect -> handshake -> ext handshake/unchoke/interested ->
// requestChunk with one in-flight request under a per-peer mutex) and src/peer_pool.zig:1-154
// (IPv4-only map, double-checked connect, evictOne can free an in-use peer).  Here: IPv4+IPv6,
// deadlines on every read, `request_many` pipelines N CHUNK_REQUESTs and matches responses by
// req_id (the reference's dead sendChunkRequests/receiveChunkResponse path), and
// pooled sessions are shared_ptr-owned so eviction never frees a session another thread uses.
#pragma once

#include <array>
#include <functional>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "bt_wire.h"
#include "net.h"
#include "sha1.h"

namespace zest::bt {

// Caller-provided destination for a response payload of n bytes (nullptr = use `data`).
using PayloadSink = std::function<uint8_t*(size_t n)>;

struct ChunkResult {
  Bytes data;
  uint32_t chunk_offset = 0;  // first chunk index of the payload inside the xorb
  std::string peer;           // address of the serving peer (for scoring / banning)
  uint8_t* ext = nullptr;     // payload landed in the request's sink instead of `data`
  size_t ext_len = 0;
  const uint8_t* bytes() const { return ext ? ext : data.data(); }
  size_t size() const { return ext ? ext_len : data.size(); }
};

struct XetRequest {
  std::array<uint8_t, 32> xorb_hash{};
  uint32_t range_start = 0, range_end = 0;
  PayloadSink sink;  // optional: receive the payload straight into caller memory (e.g. pinned)
};

class PeerSession {
 public:
  static std::shared_ptr<PeerSession> connect(const net::Addr& addr, const Sha1Digest& info_hash,
                                              const peer_id::PeerId& me, uint16_t listen_port, int timeout_ms);
  bool supports_xet() const { return remote_xet_id_ > 0; }
  const net::Addr& addr() const { return addr_; }
  const peer_id::PeerId& remote_id() const { return remote_id_; }
  std::string client() const { return client_; }
  // One request; throws Error("ChunkNotFound" | "ChunkError" | "Timeout" | ...).
  ChunkResult request(const XetRequest& r, int timeout_ms);
  // Pipelined requests; results[i] is empty + errors[i] set when that request failed.
  std::vector<ChunkResult> request_many(const std::vector<XetRequest>& reqs, int timeout_ms,
                                        std::vector<std::string>* errors = nullptr);
  bool healthy() const { return healthy_; }
  uint64_t bytes_received() const { return bytes_rx_; }
  int users() const { return users_.load(std::memory_order_relaxed); }

 private:
  PeerSession() = default;
  void read_frame(Bytes& frame, Message& m, int timeout_ms);
  net::Socket sock_;
  net::Addr addr_;
  peer_id::PeerId remote_id_{};
  int remote_xet_id_ = -1;
  std::string client_;
  uint32_t next_req_ = 1;
  bool healthy_ = true;
  uint64_t bytes_rx_ = 0;
  std::mutex mu_;  // one conversation at a time per connection
  std::atomic<int> users_{0};  // pool leases currently holding this session
  friend class PeerPool;
};

// Up to `per_peer` connections per peer address (the reference keeps one per peer and holds its
// mutex for a whole round trip, so one peer serves one request at a time — SURVEY §2.E P4).  A
// caller gets a lease: the returned pointer keeps the session's user count raised until the last
// copy is dropped, and get_or_connect hands out the least-used session, opening another
// connection while every existing one is busy.
class PeerPool {
 public:
  PeerPool(const peer_id::PeerId& me, uint16_t listen_port, size_t max_peers, int connect_timeout_ms,
           size_t per_peer = 8)
      : me_(me), listen_port_(listen_port), max_(max_peers), timeout_(connect_timeout_ms),
        per_peer_(per_peer ? per_peer : 1) {}
  // Connection reuse across info_hashes, like the reference (peer_pool.zig:4-6).
  std::shared_ptr<PeerSession> get_or_connect(const net::Addr& a, const Sha1Digest& info_hash);
  void remove(const net::Addr& a);
  size_t count() const;                         // open sessions
  size_t count(const net::Addr& a) const;       // open sessions to one peer

 private:
  std::shared_ptr<PeerSession> lease(const std::shared_ptr<PeerSession>& s);
  void evict_idle_locked(const std::string& keep);
  size_t total_locked() const;
  peer_id::PeerId me_;
  uint16_t listen_port_;
  size_t max_;
  int timeout_;
  size_t per_peer_;
  mutable std::mutex mu_;
  std::map<std::string, std::vector<std::shared_ptr<PeerSession>>> peers_;
};

}  // namespace zest::bt
