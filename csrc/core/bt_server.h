// BitTorrent seeding server: accepts peers, speaks BEP 10 + BEP XET, serves xorb ranges from a
// pluggable piece provider (HBM arena / RAM) and the disk xorb cache.
//
// Reference: src/server.zig:1-260 — listen with reuse_address (:45-80), one task per peer,
// handshake echoing the peer's info_hash, ext handshake + unchoke + interested (:113-155),
// serve loop, handleChunkRequest: chunk cache -> xorb cache getWithRange -> NOT_FOUND (:187-215),
// atomics active_peers / chunks_served.  Fixed here: responses use the *peer's* ut_xet id (the
// reference hard-codes 1), range_end is honoured by slicing full xorbs to the requested chunk run,
// the listener is closed once, and a fault injector (ZEST_FAULT) exercises the client's fallback.
#pragma once

#include <array>
#include <atomic>
#include <chrono>
#include <functional>
#include <list>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "config.h"
#include "net.h"
#include "storage.h"

namespace zest::bt {

// Returns the bytes of chunks [range_start, range_end) (or a superset starting at chunk_offset).
using PieceProvider = std::function<std::optional<storage::CacheHit>(
    const std::array<uint8_t, 32>& xorb_hash, const std::string& xet_hex, uint32_t range_start, uint32_t range_end)>;

struct ServerStats {
  uint64_t active_peers = 0;
  uint64_t total_peers = 0;
  uint64_t chunks_served = 0;
  uint64_t bytes_served = 0;
  uint64_t not_found = 0;
  uint64_t chunk_units = 0;  // Xet chunks delivered (sum of requested range lengths)
  uint64_t rejected = 0;     // connections closed at accept: max_inbound already being served
  // Where a response's time goes, summed over connections (ns): the piece provider (lookup; for
  // the HBM seeder: queueing its D2H copies), waiting for provider bytes to land (ready()), and the
  // socket writes.
  uint64_t lookup_ns = 0, wait_ns = 0, send_ns = 0;
};

struct FaultSpec {
  double drop = 0, corrupt = 0;
  int delay_ms = 0;
  // Uplink cap of the whole server in MB/s (0: none), shared by all its connections: emulates a
  // peer behind a LAN NIC (rate:1250 ~ 10 Gbps) on loopback, where striping across peers has to
  // add bandwidth.
  double rate_mbps = 0;
  static FaultSpec parse(const std::string& s);  // "drop:0.1,corrupt:0.05,delay:20,rate:1250"
};

class BtServer {
 public:
  BtServer(const Config& cfg, storage::XorbCache* cache, PieceProvider provider = {}, int port = -1);
  ~BtServer();
  void start();
  void stop();
  uint16_t port() const { return port_; }
  ServerStats stats() const;
  void set_fault(const FaultSpec& f) { fault_ = f; }

 private:
  void accept_loop();
  void handle(net::Socket s, net::Addr peer);
  std::optional<storage::CacheHit> lookup(const std::array<uint8_t, 32>& hash, uint32_t start, uint32_t end);

  const Config& cfg_;
  storage::XorbCache* cache_;
  PieceProvider provider_;
  net::Socket listener_;
  uint16_t port_ = 0;
  struct Worker {
    std::thread thread;
    std::shared_ptr<std::atomic<bool>> done;
  };
  void reap_locked();  // join finished connection threads (mu_ held)

  std::atomic<bool> stop_{false};
  std::mutex stop_mu_;  // serializes stop(): a second caller returns only after the first finished
  bool stopped_ = false;
  std::thread acceptor_;
  std::mutex mu_;
  std::set<int> conns_;
  std::list<Worker> workers_;
  std::atomic<uint64_t> active_{0}, total_{0}, served_{0}, bytes_{0}, nf_{0}, units_{0}, rejected_{0};
  std::atomic<uint64_t> lookup_ns_{0}, wait_ns_{0}, send_ns_{0};
  FaultSpec fault_;
  // rate cap: the time the uplink is free again (token bucket of one burst, shared by connections)
  std::mutex rate_mu_;
  std::chrono::steady_clock::time_point rate_free_{};
  void pace(size_t bytes);  // wait for the uplink slot of `bytes` (rate_mbps > 0)
};

// Slice chunk run [start, end) out of a serialized xorb/partial whose first chunk is `offset`.
std::optional<storage::CacheHit> slice_chunks(const Bytes& data, uint32_t offset, uint32_t start, uint32_t end);

}  // namespace zest::bt
