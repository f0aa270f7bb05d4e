#include "swarm.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <set>
#include <iomanip>

#include "trace.h"
#include "tracker.h"

namespace zest {

SwarmDownloader::SwarmDownloader(const Config& cfg, std::optional<std::string> tracker_url, bool enable_p2p,
                                 bool enable_dht, std::vector<net::Addr> dht_bootstrap)
    : cfg_(cfg), enabled_(enable_p2p), tracker_(std::move(tracker_url)) {
  if (const char* v = std::getenv("ZEST_PEER_MISS_DECAY_S"))
    miss_decay_ = std::chrono::milliseconds(int64_t(std::max(0.0, std::atof(v)) * 1000));
  pool_ = std::make_unique<bt::PeerPool>(cfg.peer_id, cfg.listen_port, cfg.max_peers, cfg.connect_timeout_ms,
                                         cfg.peer_connections);
  if (enable_p2p && enable_dht) {
    dht_ = std::make_unique<dht::Dht>(cfg.dht_port);
    if (!dht_->has_socket()) dht_ = std::make_unique<dht::Dht>(0);  // port taken: ephemeral
    dht_->start();
    if (!dht_bootstrap.empty()) {
      dht_->bootstrap(dht_bootstrap, 1500);  // explicit nodes: synchronous, so discovery can use them at once
    } else if (!cfg.dht_routers.empty()) {
      // Default public routers: resolved and queried in the background with deadlines, so an
      // offline machine pays nothing and a pull never waits on DNS (the reference lists these
      // routers but never bootstraps, leaving its DHT inert: SURVEY §2.A #7).
      boot_thread_ = std::thread([this] { bootstrap_default(); });
    }
    aq_thread_ = std::thread([this] { announce_worker(); });
  }
}

SwarmDownloader::~SwarmDownloader() {
  {
    std::lock_guard<std::mutex> g(aq_mu_);
    aq_stop_ = true;
  }
  aq_cv_.notify_all();
  if (aq_thread_.joinable()) aq_thread_.join();
  if (boot_thread_.joinable()) boot_thread_.join();
  if (dht_) dht_->stop();
}

void SwarmDownloader::bootstrap_default() {
  for (const std::string& r : cfg_.dht_routers) {
    {
      std::lock_guard<std::mutex> g(aq_mu_);
      if (aq_stop_) return;
    }
    auto a = net::resolve_with_deadline(r, 6881, 1500);
    if (!a) {
      ZTRACE("dht", "bootstrap router " << r << " did not resolve");
      continue;
    }
    const size_t n = dht_->bootstrap({*a}, 1500);
    ZTRACE("dht", "bootstrap via " << r << " (" << a->str() << "): routing table " << n);
    if (n >= 8) break;  // enough to start iterative lookups
  }
  boot_done_ = true;
}

void SwarmDownloader::announce_worker() {
  std::unique_lock<std::mutex> lk(aq_mu_);
  while (true) {
    aq_cv_.wait(lk, [&] { return aq_stop_ || !announce_q_.empty(); });
    if (aq_stop_) return;
    std::vector<Sha1Digest> batch;
    batch.swap(announce_q_);
    lk.unlock();
    for (auto& ih : batch) {
      if (dht_->table().size() == 0) break;
      try {
        dht_->announce_peer(ih, cfg_.listen_port, 1000);
      } catch (...) {
      }
      std::lock_guard<std::mutex> g(aq_mu_);
      if (aq_stop_) return;
    }
    lk.lock();
  }
}

void SwarmDownloader::add_direct_peer(const net::Addr& a) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& d : direct_)
    if (d == a) return;
  direct_.push_back(a);
}

std::vector<net::Addr> SwarmDownloader::discover(const Sha1Digest& ih) {
  const std::string key(reinterpret_cast<const char*>(ih.data()), 20);
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = discovered_.find(key);
    if (it != discovered_.end() &&
        std::chrono::steady_clock::now() - it->second.at < std::chrono::seconds(cfg_.discovery_ttl_s))
      return it->second.peers;
  }
  std::lock_guard<std::mutex> dg(disc_mu_);  // one discovery at a time (swarm.zig:320-355)
  // The first lookup waits (bounded) for the background bootstrap from the default routers.
  for (int i = 0; dht_ && i < 300 && !bootstrap_done(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  std::vector<net::Addr> peers;
  if (dht_ && dht_->table().size() > 0) {
    stats_.dht_lookups++;
    for (auto& p : dht_->get_peers(ih, 2000)) peers.push_back(p);
  }
  if (tracker_) {
    try {
      stats_.tracker_announces++;
      auto r = tracker::announce(*tracker_, ih, cfg_.peer_id, cfg_.listen_port, tracker::Event::Started, 5000);
      for (auto& p : r.peers) peers.push_back(p);
    } catch (const Error&) {
    }
  }
  std::lock_guard<std::mutex> g(mu_);
  discovered_[key] = {peers, std::chrono::steady_clock::now()};
  return peers;
}

void SwarmDownloader::remember(const net::Addr& a) {
  if (known_keys_.insert(a.str()).second) known_.push_back(a);
}

std::map<std::string, uint64_t> SwarmDownloader::peer_bytes() const {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, uint64_t> out;
  for (const auto& [k, l] : load_)
    if (l.bytes) out[k] = l.bytes;
  return out;
}

// Peers are tried in two rounds: first the direct peers plus every peer this session already knows
// (served something, or was discovered for another xorb: one seeder usually holds the whole repo),
// then -- only if none of them had the range -- the per-xorb DHT / tracker discovery.  Within a
// round the terms are striped: each attempt picks the untried candidate with the fewest requests in
// flight (peers that keep answering NOT_FOUND sink to the back), starting from a rotation by the
// xorb hash so equally loaded peers share the load evenly.  With k seeders and 16 term workers every
// seeder serves ~1/k of the bytes.  The reference runs discovery for every xorb behind one lock and
// tries peers in fixed order (swarm.zig:363-394).
std::optional<bt::ChunkResult> SwarmDownloader::try_peers(const xet::Hash& hash, uint32_t start, uint32_t end,
                                                          const bt::PayloadSink& sink) {
  if (!enabled_) return std::nullopt;
  const Sha1Digest ih = peer_id::info_hash(hash.data());
  bt::XetRequest req;
  std::memcpy(req.xorb_hash.data(), hash.data(), 32);
  req.range_start = start;
  req.range_end = end;
  req.sink = sink;
  uint64_t h0 = 0;
  std::memcpy(&h0, hash.data(), 8);
  const uint64_t rot = h0 ^ (uint64_t(start) * 0x9E3779B97F4A7C15ull);
  std::set<std::string> tried;
  // Pick the best untried candidate and count the request against it, under one lock.
  auto pick = [&](const std::vector<net::Addr>& cands) -> std::optional<net::Addr> {
    std::lock_guard<std::mutex> g(mu_);
    const size_t n = cands.size();
    std::optional<size_t> best;
    std::pair<int, int> best_key{0, 0};
    for (size_t j = 0; j < n; ++j) {
      const net::Addr& a = cands[(rot + j) % n];
      const std::string key = a.str();
      if (tried.count(key)) continue;
      auto sc = score_.find(key);
      if (sc != score_.end() && sc->second >= 3) continue;  // banned / repeatedly failing
      PeerLoad& l = load_[key];
      const auto now = std::chrono::steady_clock::now();
      if (now - l.window >= miss_decay_) {  // a new window: old NOT_FOUNDs no longer count
        l.misses = 0;
        l.window = now;
      }
      // a discovered peer that answered NOT_FOUND far more often than it served (in this window)
      // holds little of this repo: skip it (direct peers, named by the user, are always tried)
      if (l.misses >= 8 && l.misses > 4 * (l.hits + 1) && std::find(direct_.begin(), direct_.end(), a) == direct_.end())
        continue;
      const std::pair<int, int> k{l.misses > l.hits + 2 ? 1 : 0, l.inflight};
      if (!best || k < best_key) {
        best = (rot + j) % n;
        best_key = k;
      }
    }
    if (!best) return std::nullopt;
    const net::Addr& a = cands[*best];
    tried.insert(a.str());
    load_[a.str()].inflight++;
    return a;
  };
  auto attempt = [&](const std::vector<net::Addr>& cands) -> std::optional<bt::ChunkResult> {
    while (auto pa = pick(cands)) {
      const net::Addr a = *pa;
      const std::string key = a.str();
      bool hit = false, miss = false;
      uint64_t got = 0;
      std::optional<bt::ChunkResult> out;
      // the request counted by pick() is released on every path, exceptions of any type included
      struct Release {
        SwarmDownloader* self;
        const std::string& key;
        bool& hit;
        bool& miss;
        uint64_t& got;
        const net::Addr& a;
        ~Release() {
          std::lock_guard<std::mutex> g(self->mu_);
          PeerLoad& l = self->load_[key];
          l.inflight--;
          l.bytes += got;
          l.hits += hit;
          l.misses += miss;
          if (hit) {
            if (self->served_by_.insert(key).second) self->stats_.peers_connected++;
            self->remember(a);
          }
        }
      } release{this, key, hit, miss, got, a};
      try {
        auto s = pool_->get_or_connect(a, ih);
        if (s->supports_xet()) {
          trace::Span sp("peer", "request");
          bt::ChunkResult r = s->request(req, cfg_.io_timeout_ms);
          r.peer = key;
          hit = true;
          got = r.size();
          ZTRACE("swarm", "peer " << r.peer << " served " << xet::to_hex(hash) << " [" << start << "," << end
                                  << ") offset " << r.chunk_offset << " bytes " << r.size());
          stats_.peer_xorbs++;
          stats_.peer_bytes += r.size();
          stats_.total_bytes += r.size();
          stats_.total_xorbs++;
          if (dht_) {
            {
              std::lock_guard<std::mutex> g(aq_mu_);
              announce_q_.push_back(ih);
            }
            aq_cv_.notify_one();
          }
          out = std::move(r);
        }
      } catch (const Error& e) {
        stats_.peer_failures++;
        ZTRACE("swarm", "peer " << key << " failed " << xet::to_hex(hash) << " [" << start << "," << end
                                << "): " << e.what());
        if (e.code() == "ChunkNotFound" || e.code() == "ChunkError") {
          miss = true;
        } else {
          pool_->remove(a);
          std::lock_guard<std::mutex> g(mu_);
          score_[key]++;
        }
      } catch (const std::exception& e) {  // system_error / bad_alloc from connect or request
        stats_.peer_failures++;
        ZTRACE("swarm", "peer " << key << " failed " << xet::to_hex(hash) << ": " << e.what());
        pool_->remove(a);
        std::lock_guard<std::mutex> g(mu_);
        score_[key]++;
      }
      if (out) return out;
    }
    return std::nullopt;
  };
  std::vector<net::Addr> first;
  {
    std::lock_guard<std::mutex> g(mu_);
    first = direct_;
    for (const auto& k : known_)
      if (std::find(first.begin(), first.end(), k) == first.end()) first.push_back(k);
  }
  if (auto r = attempt(first)) return r;
  if (!dht_ && !tracker_) return std::nullopt;
  const std::vector<net::Addr> found = discover(ih);
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& a : found) remember(a);  // striping candidates for the following xorbs too
  }
  return attempt(found);
}

void SwarmDownloader::report_bad_peer(const std::string& addr) {
  try {
    pool_->remove(net::Addr::parse(addr));
  } catch (const Error&) {
  }
  std::lock_guard<std::mutex> g(mu_);
  score_[addr] = 1000;
  stats_.peers_banned++;
}

void SwarmDownloader::announce(const std::vector<xet::Hash>& xorbs) {
  for (const auto& h : xorbs) {
    const Sha1Digest ih = peer_id::info_hash(h.data());
    if (dht_ && dht_->table().size() > 0) dht_->announce_peer(ih, cfg_.listen_port, 1000);
    if (tracker_) {
      try {
        tracker::announce(*tracker_, ih, cfg_.peer_id, cfg_.listen_port, tracker::Event::Started, 5000);
        stats_.tracker_announces++;
      } catch (const Error&) {
      }
    }
  }
}

void SwarmDownloader::print_stats(std::ostream& w) const {
  w << "\nDownload stats:\n";
  w << "  Total xorbs:     " << stats_.total_xorbs.load() << "\n";
  w << "  From cache:      " << stats_.cached_xorbs.load() << "\n";
  w << "  From peers:      " << stats_.peer_xorbs.load() << "\n";
  w << "  From CDN:        " << stats_.cdn_xorbs.load() << "\n";
  w << "  Total bytes:     " << stats_.total_bytes.load() << "\n";
  w << "  Peers connected: " << stats_.peers_connected.load() << "\n";
  w << "  DHT lookups:     " << stats_.dht_lookups.load() << "\n";
  if (stats_.total_bytes.load() > 0) {
    const double pct = double(stats_.peer_bytes.load()) / double(stats_.total_bytes.load()) * 100.0;
    w << "  P2P ratio:       " << std::fixed << std::setprecision(1) << pct << "%\n";
  }
  const auto per_peer = peer_bytes();
  if (per_peer.size() > 1)
    for (const auto& [addr, b] : per_peer) w << "  Peer " << addr << ": " << b << " bytes\n";
}

}  // namespace zest
