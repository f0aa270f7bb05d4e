#include "bt_server.h"

#include "trace.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <random>

#include "bt_wire.h"
#include "xet_hash.h"
#include "xorb.h"

namespace zest::bt {

FaultSpec FaultSpec::parse(const std::string& s) {
  FaultSpec f;
  size_t p = 0;
  while (p < s.size()) {
    size_t c = s.find(',', p);
    std::string kv = s.substr(p, c == std::string::npos ? std::string::npos : c - p);
    size_t colon = kv.find(':');
    if (colon != std::string::npos) {
      std::string k = kv.substr(0, colon), v = kv.substr(colon + 1);
      if (k == "drop") f.drop = std::atof(v.c_str());
      else if (k == "corrupt") f.corrupt = std::atof(v.c_str());
      else if (k == "delay") f.delay_ms = std::atoi(v.c_str());
      else if (k == "rate") f.rate_mbps = std::max(0.0, std::atof(v.c_str()));
    }
    if (c == std::string::npos) break;
    p = c + 1;
  }
  return f;
}

std::optional<storage::CacheHit> slice_chunks(const Bytes& data, uint32_t offset, uint32_t start, uint32_t end) {
  return storage::slice_run(data, offset, start, end);
}

BtServer::BtServer(const Config& cfg, storage::XorbCache* cache, PieceProvider provider, int port)
    : cfg_(cfg), cache_(cache), provider_(std::move(provider)) {
  listener_ = net::Socket::listen_tcp(net::Addr::any(port < 0 ? cfg.listen_port : uint16_t(port)));
  port_ = listener_.local_addr().port();
  if (!cfg.fault.empty()) fault_ = FaultSpec::parse(cfg.fault);
}

BtServer::~BtServer() { stop(); }

void BtServer::start() {
  stop_ = false;
  acceptor_ = std::thread([this] { accept_loop(); });
}

// Safe to call from several threads at once (the REST API's /v1/stop handler and the owner's
// shutdown path both do): the TSan build caught the owner destroying the worker list while the
// API's stop() was still joining it.
void BtServer::stop() {
  std::lock_guard<std::mutex> sg(stop_mu_);
  if (stopped_) return;
  stop_ = true;
  listener_.shutdown();
  if (acceptor_.joinable()) acceptor_.join();
  std::list<Worker> ws;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    ws.swap(workers_);
  }
  for (auto& w : ws)
    if (w.thread.joinable()) w.thread.join();
  listener_.close();  // closed exactly once (server.zig double-closes)
  stopped_ = true;
}

void BtServer::reap_locked() {
  for (auto it = workers_.begin(); it != workers_.end();) {
    if (it->done->load()) {
      it->thread.join();
      it = workers_.erase(it);
    } else {
      ++it;
    }
  }
}

ServerStats BtServer::stats() const {
  ServerStats s;
  s.active_peers = active_.load();
  s.total_peers = total_.load();
  s.chunks_served = served_.load();
  s.bytes_served = bytes_.load();
  s.not_found = nf_.load();
  s.chunk_units = units_.load();
  s.rejected = rejected_.load();
  s.lookup_ns = lookup_ns_.load();
  s.wait_ns = wait_ns_.load();
  s.send_ns = send_ns_.load();
  return s;
}

void BtServer::accept_loop() {
  while (!stop_) {
    net::Addr peer;
    net::Socket s;
    try {
      s = listener_.accept(200, &peer);
    } catch (const Error&) {
      if (stop_) return;
      continue;
    }
    std::lock_guard<std::mutex> g(mu_);
    reap_locked();  // a long-running seeder must not accumulate one finished thread per connection
    if (!s.valid()) continue;
    // Every connection is served by its own thread: past max_inbound (ZEST_MAX_INBOUND) a new peer
    // is closed at once, so a flood of connections cannot exhaust threads or file descriptors (the
    // reference's server.zig accepts without bound).  The peer sees EOF and moves on.
    if (cfg_.max_inbound && conns_.size() >= cfg_.max_inbound) {
      rejected_++;
      continue;  // `s` closes here
    }
    conns_.insert(s.fd());
    auto done = std::make_shared<std::atomic<bool>>(false);
    std::thread t([this, sock = std::move(s), peer, done]() mutable {
      const int fd = sock.fd();
      try {
        handle(std::move(sock), peer);
      } catch (...) {
      }
      {
        std::lock_guard<std::mutex> g2(mu_);
        conns_.erase(fd);
      }
      done->store(true);
    });
    workers_.push_back(Worker{std::move(t), std::move(done)});
  }
}

std::optional<storage::CacheHit> BtServer::lookup(const std::array<uint8_t, 32>& hash, uint32_t start, uint32_t end) {
  xet::Hash h;
  std::memcpy(h.data(), hash.data(), 32);
  const std::string hex = xet::to_hex(h);
  if (provider_) {
    if (auto hit = provider_(hash, hex, start, end)) return hit;
  }
  if (!cache_) return std::nullopt;
  // Only runs that really hold [start, end) are served; otherwise NOT_FOUND lets the requester
  // move on to another peer or the CDN instead of receiving a run it cannot use.
  return cache_->find(hex, start, end);
}

void BtServer::handle(net::Socket s, net::Addr peer) {
  (void)peer;
  active_++;
  total_++;
  struct Dec {
    std::atomic<uint64_t>& a;
    ~Dec() { a--; }
  } dec{active_};
  s.set_timeout(cfg_.io_timeout_ms);
  s.set_buffers(8 << 20);
  uint8_t hs[kHandshakeLen];
  s.read_exact(hs, kHandshakeLen);
  Handshake theirs = parse_handshake(hs);
  Bytes out;
  write_handshake(out, theirs.info_hash, cfg_.peer_id);
  const std::string ext = bep_xet::make_ext_handshake(cfg_.listen_port);
  Bytes p(1 + ext.size());
  p[0] = 0;
  std::memcpy(p.data() + 1, ext.data(), ext.size());
  write_message(out, kExtended, p.data(), p.size());
  write_message(out, kUnchoke);
  write_message(out, kInterested);
  s.write_all(out.data(), out.size());
  int peer_xet = 1;  // until the peer tells us otherwise
  std::mt19937_64 rng(std::random_device{}());
  std::uniform_real_distribution<double> u01(0, 1);
  Bytes frame;
  while (!stop_) {
    if (!s.wait_readable(200)) continue;
    uint8_t lenb[4];
    s.read_exact(lenb, 4);
    const uint32_t len = load_be32(lenb);
    if (len > kMaxMessage) return;
    frame.resize(4 + size_t(len));
    std::memcpy(frame.data(), lenb, 4);
    if (len) s.read_exact(frame.data() + 4, len);
    Message m;
    parse_message(frame.data(), frame.size(), m);  // unknown ids throw -> connection closed
    if (m.keepalive || m.id != kExtended) continue;
    Extended e = parse_extended(m.payload);
    if (e.ext_id == 0) {
      auto caps = bep_xet::parse_ext_handshake(e.data);
      if (caps.ut_xet_id > 0) peer_xet = caps.ut_xet_id;
      continue;
    }
    bep_xet::Message x = bep_xet::decode(e.data);
    if (x.type != bep_xet::kChunkRequest) continue;
    if (fault_.delay_ms) std::this_thread::sleep_for(std::chrono::milliseconds(fault_.delay_ms));
    if (fault_.drop > 0 && u01(rng) < fault_.drop) return;  // injected connection drop
    std::optional<storage::CacheHit> hit;
    using clk = std::chrono::steady_clock;
    auto ns_since = [](clk::time_point t) {
      return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t).count());
    };
    {
      trace::Span sp("serve", "lookup");
      const auto t0 = clk::now();
      hit = lookup(x.hash, x.range_start, x.range_end);
      lookup_ns_ += ns_since(t0);
    }
    out.clear();
    if (!hit) {
      nf_++;
      bep_xet::encode_chunk_not_found(out, uint8_t(peer_xet), x.request_id, x.hash.data());
      s.write_all(out.data(), out.size());
      continue;
    }
    if (fault_.corrupt > 0 && u01(rng) < fault_.corrupt && hit->size()) {
      hit->materialize();
      hit->data[hit->data.size() / 2] ^= 0x5A;
    }
    bep_xet::encode_chunk_response_header(out, uint8_t(peer_xet), x.request_id, hit->chunk_offset,
                                          uint32_t(hit->size()));
    iovec iov[2] = {{out.data(), out.size()}, {const_cast<uint8_t*>(hit->bytes()), hit->size()}};
    {
      trace::Span sp("serve", "send");
      sp.arg("\"bytes\":" + std::to_string(hit->size()));
      if (fault_.rate_mbps > 0) {
        // paced in 1 MiB slices, so the connections of a capped server interleave on its "uplink"
        hit->wait_all();
        pace(out.size());
        s.write_all(out.data(), out.size());
        const uint8_t* b = hit->bytes();
        for (size_t o = 0, n = hit->size(); o < n;) {
          const size_t k = std::min<size_t>(n - o, size_t(1) << 20);
          pace(k);
          s.write_all(b + o, k);
          o += k;
        }
      } else if (hit->ready && hit->ext) {
        // slice by slice behind the provider's copies: slice k + 1 lands while slice k is sent
        constexpr size_t kSlice = size_t(8) << 20;
        const uint8_t* b = hit->bytes();
        const size_t n = hit->size();
        auto t = clk::now();
        s.write_all(out.data(), out.size());
        send_ns_ += ns_since(t);
        for (size_t o = 0; o < n;) {
          const size_t k = std::min(n - o, kSlice);
          t = clk::now();
          hit->ready(o + k);
          wait_ns_ += ns_since(t);
          t = clk::now();
          s.write_all(b + o, k);
          send_ns_ += ns_since(t);
          o += k;
        }
      } else {
        const auto t = clk::now();
        hit->wait_all();
        wait_ns_ += ns_since(t);
        const auto t1 = clk::now();
        s.writev_all(iov, 2);
        send_ns_ += ns_since(t1);
      }
    }
    served_++;
    bytes_ += hit->size();
    if (x.range_end > x.range_start) units_ += x.range_end - x.range_start;
  }
}

void BtServer::pace(size_t bytes) {
  using clock = std::chrono::steady_clock;
  const auto dur = std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(double(bytes) /
                                                                                             (fault_.rate_mbps * 1e6)));
  clock::time_point start;
  {
    std::lock_guard<std::mutex> g(rate_mu_);
    const auto now = clock::now();
    start = std::max(now, rate_free_);
    rate_free_ = start + dur;
  }
  std::this_thread::sleep_until(start);
}

}  // namespace zest::bt
