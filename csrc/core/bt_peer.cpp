#include <algorithm>
#include "bt_peer.h"
#include "trace.h"

#include <cstring>

namespace zest::bt {

void PeerSession::read_frame(Bytes& frame, Message& m, int timeout_ms) {
  trace::Span sp("peer", "read_frame");
  sock_.set_timeout(timeout_ms);
  uint8_t lenb[4];
  sock_.read_exact(lenb, 4);
  const uint32_t len = load_be32(lenb);
  if (len > kMaxMessage) throw Error("InvalidMessageSize");
  frame.resize(4 + size_t(len));
  std::memcpy(frame.data(), lenb, 4);
  if (len) sock_.read_exact(frame.data() + 4, len);
  bytes_rx_ += 4 + len;
  if (parse_message(frame.data(), frame.size(), m) == 0) throw Error("UnexpectedEnd");
}

std::shared_ptr<PeerSession> PeerSession::connect(const net::Addr& addr, const Sha1Digest& info_hash,
                                                  const peer_id::PeerId& me, uint16_t listen_port, int timeout_ms) {
  std::shared_ptr<PeerSession> s(new PeerSession());
  s->addr_ = addr;
  s->sock_ = net::Socket::connect_tcp(addr, timeout_ms);
  s->sock_.set_timeout(timeout_ms);
  s->sock_.set_buffers(8 << 20);
  Bytes out;
  write_handshake(out, info_hash, me);
  s->sock_.write_all(out.data(), out.size());
  uint8_t hs[kHandshakeLen];
  s->sock_.read_exact(hs, kHandshakeLen);
  Handshake h = parse_handshake(hs);
  if (h.info_hash != info_hash) throw Error("InfoHashMismatch");
  s->remote_id_ = h.peer_id;
  if (!h.supports_bep10()) return s;
  out.clear();
  const std::string ext = bep_xet::make_ext_handshake(listen_port);
  Bytes payload(1 + ext.size());
  payload[0] = 0;  // ext_id 0 = extended handshake
  std::memcpy(payload.data() + 1, ext.data(), ext.size());
  write_message(out, kExtended, payload.data(), payload.size());
  write_message(out, kUnchoke);
  write_message(out, kInterested);
  s->sock_.write_all(out.data(), out.size());
  // Read until the peer's extended handshake (bounded).
  Bytes frame;
  for (int i = 0; i < 8; ++i) {
    Message m;
    s->read_frame(frame, m, timeout_ms);
    if (m.keepalive || m.id != kExtended) continue;
    Extended e = parse_extended(m.payload);
    if (e.ext_id != 0) continue;
    bep_xet::ExtCapabilities caps = bep_xet::parse_ext_handshake(e.data);
    s->remote_xet_id_ = caps.ut_xet_id;
    s->client_ = caps.client;
    break;
  }
  return s;
}

ChunkResult PeerSession::request(const XetRequest& r, int timeout_ms) {
  std::vector<std::string> errs;
  auto res = request_many({r}, timeout_ms, &errs);
  if (!errs[0].empty()) throw Error(errs[0]);
  return std::move(res[0]);
}

std::vector<ChunkResult> PeerSession::request_many(const std::vector<XetRequest>& reqs, int timeout_ms,
                                                   std::vector<std::string>* errors) {
  std::lock_guard<std::mutex> g(mu_);
  if (!supports_xet()) throw Error("PeerNoXet");
  std::vector<ChunkResult> out(reqs.size());
  std::vector<std::string> errs(reqs.size());
  std::map<uint32_t, size_t> want;
  Bytes msg;
  for (size_t i = 0; i < reqs.size(); ++i) {
    const uint32_t id = next_req_++;
    want[id] = i;
    bep_xet::encode_chunk_request(msg, uint8_t(remote_xet_id_), id, reqs[i].xorb_hash.data(), reqs[i].range_start,
                                  reqs[i].range_end);
  }
  try {
    sock_.write_all(msg.data(), msg.size());
    Bytes frame;
    while (!want.empty()) {
      // Fast path: a CHUNK_RESPONSE's payload is read straight into its result buffer (one
      // kernel->user copy, no frame buffer + second copy for 64 MiB runs).
      sock_.set_timeout(timeout_ms);
      uint8_t lenb[4];
      sock_.read_exact(lenb, 4);
      const uint32_t len = load_be32(lenb);
      if (len > kMaxMessage) throw Error("InvalidMessageSize");
      constexpr uint32_t kPre = 15;  // id, ext id, type, request_id, chunk_offset, data_len
      uint8_t pre[kPre];
      uint32_t have = 0;
      if (len >= kPre) {
        sock_.read_exact(pre, kPre);
        have = kPre;
        if (pre[0] == kExtended && pre[1] != 0 && pre[2] == bep_xet::kChunkResponse &&
            load_be32(pre + 11) == len - kPre) {
          const uint32_t rid = load_be32(pre + 3), dlen = len - kPre;
          auto it = want.find(rid);
          bytes_rx_ += 4 + len;
          if (it == want.end()) {  // stale reply: drain it
            frame.resize(dlen);
            if (dlen) sock_.read_exact(frame.data(), dlen);
            continue;
          }
          const size_t i = it->second;
          want.erase(it);
          trace::Span sp("peer", "read_payload");
          uint8_t* dst = reqs[i].sink ? reqs[i].sink(dlen) : nullptr;
          if (dst) {
            out[i].ext = dst;
            out[i].ext_len = dlen;
          } else {
            out[i].data.resize(dlen);
            dst = out[i].data.data();
          }
          if (dlen) sock_.read_exact(dst, dlen);
          out[i].chunk_offset = load_be32(pre + 7);
          continue;
        }
      }
      frame.resize(4 + size_t(len));
      std::memcpy(frame.data(), lenb, 4);
      std::memcpy(frame.data() + 4, pre, have);
      if (len > have) sock_.read_exact(frame.data() + 4 + have, len - have);
      bytes_rx_ += 4 + len;
      Message m;
      if (parse_message(frame.data(), frame.size(), m) == 0) throw Error("UnexpectedEnd");
      if (m.keepalive) continue;
      if (m.id == kChoke || m.id == kUnchoke || m.id == kInterested || m.id == kNotInterested) continue;
      if (m.id != kExtended) continue;
      Extended e = parse_extended(m.payload);
      if (e.ext_id == 0) continue;  // late/extra ext handshake
      bep_xet::Message x = bep_xet::decode(e.data);
      auto it = want.find(x.request_id);
      if (it == want.end()) continue;  // stale reply for another request
      const size_t i = it->second;
      want.erase(it);
      switch (x.type) {
        case bep_xet::kChunkResponse:
          out[i].data.assign(x.data.data, x.data.data + x.data.size);
          out[i].chunk_offset = x.chunk_offset;
          break;
        case bep_xet::kChunkNotFound: errs[i] = "ChunkNotFound"; break;
        case bep_xet::kChunkError: errs[i] = "ChunkError"; break;
        default: errs[i] = "UnexpectedMessage"; break;
      }
    }
  } catch (const Error&) {
    healthy_ = false;
    throw;
  }
  if (errors) *errors = std::move(errs);
  return out;
}

std::shared_ptr<PeerSession> PeerPool::lease(const std::shared_ptr<PeerSession>& s) {
  // Constructed in place and non-copyable: the count is raised once and dropped once.  (A
  // temporary `Lease{s}` copied into make_shared ran the destructor twice, so every finished
  // request left its session one below zero, and "least used" then sent every later request to
  // the one session used most -- all workers queued on a single connection.)
  struct Lease {
    explicit Lease(std::shared_ptr<PeerSession> p) : s(std::move(p)) { s->users_.fetch_add(1, std::memory_order_relaxed); }
    Lease(const Lease&) = delete;
    Lease& operator=(const Lease&) = delete;
    ~Lease() { s->users_.fetch_sub(1, std::memory_order_relaxed); }
    std::shared_ptr<PeerSession> s;
  };
  auto l = std::make_shared<Lease>(s);
  return std::shared_ptr<PeerSession>(l, s.get());  // aliasing: lives as long as the lease
}

size_t PeerPool::total_locked() const {
  size_t n = 0;
  for (const auto& [k, v] : peers_) n += v.size();
  return n;
}

void PeerPool::evict_idle_locked(const std::string& keep) {
  for (auto it = peers_.begin(); it != peers_.end() && total_locked() >= max_;) {
    auto& v = it->second;
    if (it->first != keep)
      v.erase(std::remove_if(v.begin(), v.end(), [](const auto& s) { return s->users() == 0 && s.use_count() == 1; }),
              v.end());
    it = v.empty() ? peers_.erase(it) : std::next(it);
  }
}

std::shared_ptr<PeerSession> PeerPool::get_or_connect(const net::Addr& a, const Sha1Digest& info_hash) {
  const std::string key = a.str();
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& v = peers_[key];
    v.erase(std::remove_if(v.begin(), v.end(), [](const auto& s) { return !s->healthy(); }), v.end());
    std::shared_ptr<PeerSession> best;
    for (auto& s : v)
      if (!best || s->users() < best->users()) best = s;
    if (best && (best->users() == 0 || v.size() >= per_peer_)) return lease(best);
  }
  // Every session to this peer is busy (or there is none): connect + handshake outside the lock.
  auto s = PeerSession::connect(a, info_hash, me_, listen_port_, timeout_);
  std::lock_guard<std::mutex> g(mu_);
  auto& v = peers_[key];
  if (v.size() >= per_peer_) {  // others connected meanwhile: use the least-used one
    std::shared_ptr<PeerSession> best;
    for (auto& x : v)
      if (x->healthy() && (!best || x->users() < best->users())) best = x;
    if (best) return lease(best);
  }
  if (total_locked() >= max_) evict_idle_locked(key);
  peers_[key].push_back(s);
  return lease(s);
}

void PeerPool::remove(const net::Addr& a) {
  std::lock_guard<std::mutex> g(mu_);
  peers_.erase(a.str());
}

size_t PeerPool::count() const {
  std::lock_guard<std::mutex> g(mu_);
  return total_locked();
}

size_t PeerPool::count(const net::Addr& a) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = peers_.find(a.str());
  return it == peers_.end() ? 0 : it->second.size();
}

}  // namespace zest::bt
