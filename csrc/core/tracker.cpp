#include "tracker.h"

#include <arpa/inet.h>

#include <cstring>

#include "bencode.h"
#include "http.h"

namespace zest::tracker {

const char* event_str(Event e) {
  switch (e) {
    case Event::Started: return "started";
    case Event::Stopped: return "stopped";
    case Event::Completed: return "completed";
    default: return nullptr;
  }
}

std::string announce_url(const std::string& tracker_url, const Sha1Digest& ih, const peer_id::PeerId& pid,
                         uint16_t port, Event ev, uint64_t uploaded, uint64_t downloaded, uint64_t left) {
  std::string u = tracker_url;
  while (!u.empty() && u.back() == '/') u.pop_back();
  if (u.size() < 9 || u.compare(u.size() - 9, 9, "/announce") != 0) u += "/announce";
  u += (u.find('?') == std::string::npos ? "?" : "&");
  u += "info_hash=" + http::percent_encode(ih.data(), 20);
  u += "&peer_id=" + http::percent_encode(pid.data(), 20);
  u += "&port=" + std::to_string(port);
  u += "&compact=1&uploaded=" + std::to_string(uploaded) + "&downloaded=" + std::to_string(downloaded) +
       "&left=" + std::to_string(left);
  if (const char* e = event_str(ev)) u += std::string("&event=") + e;
  return u;
}

std::vector<net::Addr> parse_compact_peers(std::string_view d, bool v6) {
  std::vector<net::Addr> out;
  const size_t rec = v6 ? 18 : 6;
  if (d.size() % rec != 0) return out;
  for (size_t i = 0; i < d.size(); i += rec) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(d.data() + i);
    if (!v6) {
      out.push_back(net::Addr::ipv4(p, uint16_t((p[4] << 8) | p[5])));
    } else {
      net::Addr a;
      sockaddr_in6 s6{};
      s6.sin6_family = AF_INET6;
      std::memcpy(&s6.sin6_addr, p, 16);
      s6.sin6_port = htons(uint16_t((p[16] << 8) | p[17]));
      std::memcpy(&a.ss, &s6, sizeof(s6));
      a.len = sizeof(s6);
      out.push_back(a);
    }
  }
  return out;
}

std::string encode_compact_peer(const net::Addr& a) {
  std::string s;
  if (a.is_v4()) {
    uint8_t ip[4];
    a.ipv4_bytes(ip);
    s.append(reinterpret_cast<char*>(ip), 4);
  } else {
    const auto* s6 = reinterpret_cast<const sockaddr_in6*>(&a.ss);
    s.append(reinterpret_cast<const char*>(&s6->sin6_addr), 16);
  }
  const uint16_t p = a.port();
  s.push_back(char(p >> 8));
  s.push_back(char(p & 0xFF));
  return s;
}

AnnounceResponse parse_announce(std::string_view body) {
  bencode::Document doc;
  doc.parse(body);
  bencode::Ref root = doc.root();
  if (!root.is_dict()) throw Error("InvalidFormat", "tracker response is not a dict");
  if (bencode::Ref f = root.get("failure reason"); f.is_str()) throw Error("TrackerError", std::string(f.as_str()));
  AnnounceResponse r;
  const int64_t iv = root.get_int("interval", 1800);
  r.interval = iv > 0 ? uint32_t(iv) : 1800;
  bencode::Ref peers = root.get("peers");
  if (peers.is_str()) {
    r.peers = parse_compact_peers(peers.as_str(), false);
  } else if (peers.is_list()) {
    for (bencode::Ref p : peers.children()) {
      if (!p.is_dict()) continue;
      std::string_view ip = p.get_str("ip");
      int64_t port = p.get_int("port", 0);
      if (ip.empty() || port <= 0 || port > 65535) continue;
      try {
        r.peers.push_back(net::Addr::resolve(ip, uint16_t(port)));
      } catch (const Error&) {
      }
    }
  }
  if (bencode::Ref p6 = root.get("peers6"); p6.is_str()) {
    auto v = parse_compact_peers(p6.as_str(), true);
    r.peers.insert(r.peers.end(), v.begin(), v.end());
  }
  return r;
}

AnnounceResponse announce(const std::string& tracker_url, const Sha1Digest& ih, const peer_id::PeerId& pid,
                          uint16_t port, Event ev, int timeout_ms) {
  http::RequestOptions opt;
  opt.timeout_ms = timeout_ms;
  opt.max_body = 1 << 20;
  http::Response resp = http::get(announce_url(tracker_url, ih, pid, port, ev), {}, opt);
  if (resp.status != 200) throw Error("HttpError", "tracker status " + std::to_string(resp.status));
  return parse_announce(resp.body);
}

}  // namespace zest::tracker
