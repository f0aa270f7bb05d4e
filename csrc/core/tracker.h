// BitTorrent HTTP tracker client (BEP 3 announce, BEP 23 compact peers, BEP 7 peers6).
//
// Reference: src/bt_tracker.zig:1-260 — GET {url}/announce?info_hash=..&peer_id=..&port=N
// &compact=1&uploaded=0&downloaded=0&left=0[&event=started] (:65-86), RFC 3986 percent-encoding
// (:110-128), bencoded `failure reason` -> TrackerError, default interval 1800 (:131-180).
// Extension over the reference: dict-model `peers` lists and `peers6` are accepted too.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "net.h"
#include "sha1.h"

namespace zest::tracker {

enum class Event { None, Started, Stopped, Completed };
const char* event_str(Event e);

struct AnnounceResponse {
  uint32_t interval = 1800;
  std::vector<net::Addr> peers;
};

std::string announce_url(const std::string& tracker_url, const Sha1Digest& info_hash, const peer_id::PeerId& pid,
                         uint16_t port, Event ev, uint64_t uploaded = 0, uint64_t downloaded = 0, uint64_t left = 0);
// Throws Error("TrackerError", reason) on `failure reason`, Error("InvalidFormat") on garbage.
AnnounceResponse parse_announce(std::string_view body);
AnnounceResponse announce(const std::string& tracker_url, const Sha1Digest& info_hash, const peer_id::PeerId& pid,
                          uint16_t port, Event ev, int timeout_ms = 10000);

// Compact peer list encoding shared with the DHT (6 bytes IPv4 + port, 18 bytes IPv6 + port).
std::vector<net::Addr> parse_compact_peers(std::string_view data, bool v6 = false);
std::string encode_compact_peer(const net::Addr& a);

}  // namespace zest::tracker
