#include "dht.h"

#include <algorithm>
#include <cstring>
#include <random>

#include "bencode.h"
#include "tracker.h"

namespace zest::dht {

NodeId xor_distance(const NodeId& a, const NodeId& b) {
  NodeId d;
  for (int i = 0; i < 20; ++i) d[i] = a[i] ^ b[i];
  return d;
}

bool closer(const NodeId& t, const NodeId& a, const NodeId& b) {
  for (int i = 0; i < 20; ++i) {
    const uint8_t da = t[i] ^ a[i], db = t[i] ^ b[i];
    if (da != db) return da < db;
  }
  return false;
}

int bucket_index(const NodeId& own, const NodeId& other) {
  for (int i = 0; i < 20; ++i) {
    const uint8_t d = own[i] ^ other[i];
    if (d) return i * 8 + __builtin_clz(uint32_t(d)) - 24;
  }
  return -1;
}

NodeId random_id() {
  NodeId id;
  std::random_device rd;
  for (auto& b : id) b = uint8_t(rd());
  return id;
}

bool RoutingTable::insert(const NodeInfo& n) {
  const int b = bucket_index(own_, n.id);
  if (b < 0) return false;
  std::lock_guard<std::mutex> g(mu_);
  auto& bk = buckets_[size_t(b)];
  for (auto& e : bk) {
    if (e.id == n.id) {
      e.addr = n.addr;
      return true;
    }
  }
  if (bk.size() >= size_t(K)) return false;
  bk.push_back(n);
  return true;
}

void RoutingTable::remove(const NodeId& id) {
  const int b = bucket_index(own_, id);
  if (b < 0) return;
  std::lock_guard<std::mutex> g(mu_);
  auto& bk = buckets_[size_t(b)];
  bk.erase(std::remove_if(bk.begin(), bk.end(), [&](const NodeInfo& e) { return e.id == id; }), bk.end());
}

std::vector<NodeInfo> RoutingTable::closest(const NodeId& target, size_t k) const {
  std::vector<NodeInfo> all;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& bk : buckets_) all.insert(all.end(), bk.begin(), bk.end());
  }
  std::sort(all.begin(), all.end(), [&](const NodeInfo& a, const NodeInfo& b) { return closer(target, a.id, b.id); });
  if (all.size() > k) all.resize(k);
  return all;
}

size_t RoutingTable::size() const {
  std::lock_guard<std::mutex> g(mu_);
  size_t n = 0;
  for (auto& bk : buckets_) n += bk.size();
  return n;
}

namespace {
std::string_view idv(const NodeId& id) { return {reinterpret_cast<const char*>(id.data()), 20}; }
std::string_view ihv(const Sha1Digest& d) { return {reinterpret_cast<const char*>(d.data()), 20}; }
}  // namespace

std::string build_ping(std::string_view tid, const NodeId& own) {
  std::string o;
  bencode::Encoder e(o);
  e.begin_dict().key("a").begin_dict().key("id").str(idv(own)).end();
  e.key("q").str("ping").key("t").str(tid).key("y").str("q").end();
  return o;
}

std::string build_find_node(std::string_view tid, const NodeId& own, const NodeId& target) {
  std::string o;
  bencode::Encoder e(o);
  e.begin_dict().key("a").begin_dict().key("id").str(idv(own)).key("target").str(idv(target)).end();
  e.key("q").str("find_node").key("t").str(tid).key("y").str("q").end();
  return o;
}

std::string build_get_peers(std::string_view tid, const NodeId& own, const Sha1Digest& ih) {
  std::string o;
  bencode::Encoder e(o);
  e.begin_dict().key("a").begin_dict().key("id").str(idv(own)).key("info_hash").str(ihv(ih)).end();
  e.key("q").str("get_peers").key("t").str(tid).key("y").str("q").end();
  return o;
}

std::string build_announce_peer(std::string_view tid, const NodeId& own, const Sha1Digest& ih, uint16_t port,
                                std::string_view token, bool implied_port) {
  std::string o;
  bencode::Encoder e(o);
  e.begin_dict().key("a").begin_dict();
  e.key("id").str(idv(own)).key("implied_port").integer(implied_port ? 1 : 0);
  e.key("info_hash").str(ihv(ih)).key("port").integer(port).key("token").str(token).end();
  e.key("q").str("announce_peer").key("t").str(tid).key("y").str("q").end();
  return o;
}

std::vector<NodeInfo> parse_compact_nodes(std::string_view d) {
  std::vector<NodeInfo> out;
  if (d.size() % 26 != 0) return out;
  for (size_t i = 0; i < d.size(); i += 26) {
    NodeInfo n;
    std::memcpy(n.id.data(), d.data() + i, 20);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(d.data() + i + 20);
    n.addr = net::Addr::ipv4(p, uint16_t((p[4] << 8) | p[5]));
    out.push_back(n);
  }
  return out;
}

std::string encode_compact_node(const NodeInfo& n) {
  std::string s(reinterpret_cast<const char*>(n.id.data()), 20);
  if (n.addr.is_v4()) s += tracker::encode_compact_peer(n.addr);
  else s.append(6, '\0');
  return s;
}

Dht::Dht(uint16_t port, NodeId own) : table_(own) {
  try {
    sock_ = net::Socket::udp(net::Addr::any(port));
    port_ = sock_.local_addr().port();
  } catch (const Error&) {
    port_ = 0;
  }
  std::random_device rd;
  for (int i = 0; i < 16; ++i) secret_.push_back(char(rd()));
}

Dht::~Dht() { stop(); }

void Dht::start() {
  if (!sock_.valid() || thr_.joinable()) return;
  stop_ = false;
  thr_ = std::thread([this] { recv_loop(); });
}

void Dht::stop() {
  stop_ = true;
  if (thr_.joinable()) thr_.join();
}

std::string Dht::next_tid() {
  const uint32_t t = tid_.fetch_add(1);
  std::string s(2, '\0');
  s[0] = char(t >> 8);
  s[1] = char(t);
  return s;
}

std::string Dht::token_for(const net::Addr& a) const {
  std::string m = secret_ + a.host();
  Sha1Digest d = Sha1::hash(m.data(), m.size());
  return std::string(reinterpret_cast<const char*>(d.data()), 8);
}

bool Dht::rpc(const net::Addr& to, const std::string& msg, const std::string& tid, int timeout_ms, std::string& reply) {
  if (!sock_.valid()) return false;
  {
    std::lock_guard<std::mutex> g(mu_);
    pending_[tid] = Pending{};
    stats_.queries_sent++;
  }
  try {
    sock_.send_to(to, msg.data(), msg.size());
  } catch (const Error&) {
    std::lock_guard<std::mutex> g(mu_);
    pending_.erase(tid);
    return false;
  }
  std::unique_lock<std::mutex> lk(mu_);
  const bool ok = cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return pending_[tid].done; });
  if (ok) {
    reply = std::move(pending_[tid].reply);
    stats_.responses++;
  } else {
    stats_.timeouts++;
  }
  pending_.erase(tid);
  return ok;
}

void Dht::recv_loop() {
  std::vector<uint8_t> buf(65536);
  while (!stop_) {
    net::Addr from;
    size_t n = 0;
    try {
      n = sock_.recv_from(buf.data(), buf.size(), &from, 100);
    } catch (const Error&) {
      continue;
    }
    if (n == 0) continue;
    std::string pkt(reinterpret_cast<char*>(buf.data()), n);
    try {
      bencode::Document doc;
      doc.parse(pkt);
      bencode::Ref r = doc.root();
      if (!r.is_dict()) continue;
      std::string_view y = r.get_str("y");
      if (y == "r" || y == "e") {
        std::string tid(r.get_str("t"));
        // learn the responder
        bencode::Ref body = r.get("r");
        if (body.is_dict()) {
          std::string_view id = body.get_str("id");
          if (id.size() == 20) {
            NodeInfo ni;
            std::memcpy(ni.id.data(), id.data(), 20);
            ni.addr = from;
            table_.insert(ni);
          }
        }
        std::lock_guard<std::mutex> g(mu_);
        auto it = pending_.find(tid);
        if (it != pending_.end()) {
          it->second.done = true;
          it->second.reply = pkt;
          it->second.from = from;
          cv_.notify_all();
        }
      } else if (y == "q") {
        handle_query(pkt, from);
      }
    } catch (const Error&) {
    }
  }
}

void Dht::handle_query(const std::string& pkt, const net::Addr& from) {
  bencode::Document doc;
  doc.parse(pkt);
  bencode::Ref r = doc.root();
  std::string_view q = r.get_str("q");
  std::string_view tid = r.get_str("t");
  bencode::Ref a = r.get("a");
  if (!a.is_dict()) return;
  std::string_view qid = a.get_str("id");
  if (qid.size() == 20) {
    NodeInfo ni;
    std::memcpy(ni.id.data(), qid.data(), 20);
    ni.addr = from;
    table_.insert(ni);
  }
  std::string out;
  bencode::Encoder e(out);
  auto begin_reply = [&]() { e.begin_dict().key("r").begin_dict(); };
  auto end_reply = [&]() { e.end().key("t").str(tid).key("y").str("r").end(); };
  auto nodes_of = [&](const NodeId& target) {
    std::string s;
    for (auto& n : table_.closest(target, K)) s += encode_compact_node(n);
    return s;
  };
  if (q == "ping") {
    begin_reply();
    e.key("id").str(idv(id()));
    end_reply();
  } else if (q == "find_node") {
    std::string_view t = a.get_str("target");
    if (t.size() != 20) return;
    NodeId target;
    std::memcpy(target.data(), t.data(), 20);
    begin_reply();
    e.key("id").str(idv(id())).key("nodes").str(nodes_of(target));
    end_reply();
  } else if (q == "get_peers") {
    std::string_view ih = a.get_str("info_hash");
    if (ih.size() != 20) return;
    NodeId target;
    std::memcpy(target.data(), ih.data(), 20);
    std::vector<net::Addr> peers;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = store_.find(std::string(ih));
      if (it != store_.end()) peers = it->second;
    }
    begin_reply();
    e.key("id").str(idv(id())).key("nodes").str(nodes_of(target)).key("token").str(token_for(from));
    if (!peers.empty()) {
      e.key("values").begin_list();
      for (auto& p : peers) e.str(tracker::encode_compact_peer(p));
      e.end();
    }
    end_reply();
  } else if (q == "announce_peer") {
    std::string_view ih = a.get_str("info_hash");
    if (ih.size() != 20 || a.get_str("token") != token_for(from)) {
      e.begin_dict().key("e").begin_list().integer(203).str("bad token").end();
      e.key("t").str(tid).key("y").str("e").end();
    } else {
      uint16_t port = a.get_int("implied_port", 0) ? from.port() : uint16_t(a.get_int("port", 0));
      net::Addr peer = from;
      if (peer.is_v4()) {
        uint8_t ip[4];
        peer.ipv4_bytes(ip);
        peer = net::Addr::ipv4(ip, port);
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        auto& v = store_[std::string(ih)];
        if (std::find(v.begin(), v.end(), peer) == v.end()) v.push_back(peer);
      }
      begin_reply();
      e.key("id").str(idv(id()));
      end_reply();
    }
  } else {
    e.begin_dict().key("e").begin_list().integer(204).str("method unknown").end();
    e.key("t").str(tid).key("y").str("e").end();
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    stats_.queries_answered++;
  }
  try {
    sock_.send_to(from, out.data(), out.size());
  } catch (const Error&) {
  }
}

bool Dht::ping(const net::Addr& a, int timeout_ms) {
  std::string tid = next_tid(), reply;
  return rpc(a, build_ping(tid, id()), tid, timeout_ms, reply);
}

size_t Dht::bootstrap(const std::vector<net::Addr>& nodes, int timeout_ms) {
  for (auto& n : nodes) {
    std::string tid = next_tid(), reply;
    if (!rpc(n, build_find_node(tid, id(), id()), tid, timeout_ms, reply)) continue;
    try {
      bencode::Document doc;
      doc.parse(reply);
      bencode::Ref r = doc.root().get("r");
      for (auto& ni : parse_compact_nodes(r.get_str("nodes"))) table_.insert(ni);
    } catch (const Error&) {
    }
  }
  return table_.size();
}

std::vector<net::Addr> Dht::get_peers(const Sha1Digest& ih, int timeout_ms) {
  {
    std::lock_guard<std::mutex> g(mu_);
    stats_.lookups++;
  }
  NodeId target;
  std::memcpy(target.data(), ih.data(), 20);
  std::vector<NodeInfo> shortlist = table_.closest(target, K);
  std::set<std::string> queried;
  std::vector<net::Addr> peers;
  std::vector<std::pair<net::Addr, std::string>> toks;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (std::chrono::steady_clock::now() < deadline) {
    std::vector<NodeInfo> batch;
    for (auto& n : shortlist) {
      if (queried.count(n.addr.str())) continue;
      batch.push_back(n);
      if (batch.size() >= size_t(ALPHA)) break;
    }
    if (batch.empty()) break;
    bool progress = false;
    std::vector<std::thread> ts;
    std::mutex m;
    for (auto& n : batch) {
      queried.insert(n.addr.str());
      ts.emplace_back([&, n] {
        std::string tid = next_tid(), reply;
        if (!rpc(n.addr, build_get_peers(tid, id(), ih), tid, std::min(timeout_ms, 1500), reply)) {
          table_.remove(n.id);
          return;
        }
        try {
          bencode::Document doc;
          doc.parse(reply);
          bencode::Ref r = doc.root().get("r");
          if (!r.is_dict()) return;
          std::lock_guard<std::mutex> g(m);
          if (std::string_view tok = r.get_str("token"); !tok.empty()) toks.emplace_back(n.addr, std::string(tok));
          if (bencode::Ref vals = r.get("values"); vals.is_list())
            for (auto v : vals.children())
              if (v.is_str())
                for (auto& p : tracker::parse_compact_peers(v.as_str())) peers.push_back(p);
          for (auto& ni : parse_compact_nodes(r.get_str("nodes"))) {
            table_.insert(ni);
            bool dup = false;
            for (auto& s : shortlist)
              if (s.id == ni.id) dup = true;
            if (!dup && ni.id != id()) {
              shortlist.push_back(ni);
              progress = true;
            }
          }
        } catch (const Error&) {
        }
      });
    }
    for (auto& t : ts) t.join();
    std::sort(shortlist.begin(), shortlist.end(),
              [&](const NodeInfo& a, const NodeInfo& b) { return closer(target, a.id, b.id); });
    if (shortlist.size() > size_t(2 * K)) shortlist.resize(2 * K);
    if (!progress && !peers.empty()) break;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    tokens_[std::string(ihv(ih))] = toks;
  }
  std::sort(peers.begin(), peers.end(), [](const net::Addr& a, const net::Addr& b) { return a.str() < b.str(); });
  peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
  return peers;
}

size_t Dht::announce_peer(const Sha1Digest& ih, uint16_t port, int timeout_ms) {
  std::vector<std::pair<net::Addr, std::string>> toks;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = tokens_.find(std::string(ihv(ih)));
    if (it != tokens_.end()) toks = it->second;
  }
  if (toks.empty()) {
    get_peers(ih, timeout_ms);
    std::lock_guard<std::mutex> g(mu_);
    toks = tokens_[std::string(ihv(ih))];
  }
  size_t ok = 0;
  for (auto& [addr, tok] : toks) {
    std::string tid = next_tid(), reply;
    if (rpc(addr, build_announce_peer(tid, id(), ih, port, tok), tid, std::min(timeout_ms, 1500), reply)) ++ok;
  }
  return ok;
}

DhtStats Dht::stats() const {
  std::lock_guard<std::mutex> g(mu_);
  return stats_;
}

std::vector<net::Addr> Dht::stored_peers(const Sha1Digest& ih) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = store_.find(std::string(ihv(ih)));
  return it == store_.end() ? std::vector<net::Addr>{} : it->second;
}

}  // namespace zest::dht
