// BitTorrent wire framing (BEP 3 + BEP 10) and the BEP XET extension messages.
//
// Reference: src/bt_wire.zig:1-274 (68-byte handshake with reserved byte 5 = 0x10, [u32 BE len]
// [id][payload] messages, keepalive = 4 zero bytes, extended = id 20 + ext_id, 64 MiB + 1 KiB
// cap) and src/bep_xet.zig:1-362 (ut_xet CHUNK_REQUEST 45 B / CHUNK_RESPONSE 13+N /
// CHUNK_NOT_FOUND 37 B / CHUNK_ERROR 9+N, ext handshake {"m":{"ut_xet":1},"p":port,"v":...}).
// Differences by design: unknown message ids / XET types are reported as errors instead of the
// reference's illegal @enumFromInt (bt_wire.zig:119, bep_xet.zig:132), and encoders write into
// caller buffers so a CHUNK_RESPONSE payload can be sent zero-copy (scatter write).
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>

#include "common.h"
#include "sha1.h"

namespace zest::bt {

constexpr std::string_view kProtocol = "BitTorrent protocol";
constexpr size_t kHandshakeLen = 68;
constexpr uint32_t kMaxMessage = (64u << 20) + 1024u;
constexpr uint8_t kReserved[8] = {0, 0, 0, 0, 0, 0x10, 0, 0};

enum MsgId : uint8_t {
  kChoke = 0,
  kUnchoke = 1,
  kInterested = 2,
  kNotInterested = 3,
  kHave = 4,
  kBitfield = 5,
  kRequest = 6,
  kPiece = 7,
  kCancel = 8,
  kExtended = 20,
};
bool known_msg_id(uint8_t id);

struct Handshake {
  std::array<uint8_t, 8> reserved{};
  Sha1Digest info_hash{};
  peer_id::PeerId peer_id{};
  bool supports_bep10() const { return (reserved[5] & 0x10) != 0; }
};

void write_handshake(Bytes& out, const Sha1Digest& info_hash, const peer_id::PeerId& peer_id);
Handshake parse_handshake(const uint8_t* p68);  // throws Error("InvalidProtocolString")

void write_message(Bytes& out, uint8_t id, const uint8_t* payload = nullptr, size_t n = 0);
// Fixed-buffer variant (caller guarantees 5 + n bytes of room); returns bytes written.
inline size_t write_message(uint8_t* out, uint8_t id, const uint8_t* payload, size_t n) {
  store_be32(out, uint32_t(1 + n));
  out[4] = id;
  if (n) std::memcpy(out + 5, payload, n);
  return 5 + n;
}
void write_keepalive(Bytes& out);
void write_extended(Bytes& out, uint8_t ext_id, const uint8_t* payload, size_t n);

struct Message {
  bool keepalive = false;
  uint8_t id = 0;
  ByteSpan payload;
};
// Frame parser over a receive buffer.  Returns bytes consumed (0 = need more data).
// Throws Error("InvalidMessageSize") above kMaxMessage.
size_t parse_message(const uint8_t* p, size_t n, Message& m);
// Length of the next frame if its 4-byte prefix is available (0 otherwise).
size_t frame_length(const uint8_t* p, size_t n);

struct Extended {
  uint8_t ext_id;
  ByteSpan data;
};
Extended parse_extended(ByteSpan payload);  // throws Error("UnexpectedEnd")

}  // namespace zest::bt

namespace zest::bep_xet {

constexpr std::string_view kExtName = "ut_xet";
constexpr std::string_view kClientVersion = "zest/0.4";

enum Type : uint8_t { kChunkRequest = 1, kChunkResponse = 2, kChunkNotFound = 3, kChunkError = 4 };

struct Message {
  Type type{};
  uint32_t request_id = 0;
  std::array<uint8_t, 32> hash{};  // request / not_found
  uint32_t range_start = 0, range_end = 0;  // request
  uint32_t chunk_offset = 0;  // response
  uint32_t error_code = 0;    // error
  ByteSpan data;              // response data / error message
};

// Full wire messages (length prefix + id 20 + ext_id + XET payload).
void encode_chunk_request(Bytes& out, uint8_t ext_id, uint32_t request_id, const uint8_t hash[32],
                          uint32_t range_start, uint32_t range_end);
// Header only (6 + 13 bytes); the caller sends `data_len` payload bytes right after it.
void encode_chunk_response_header(Bytes& out, uint8_t ext_id, uint32_t request_id, uint32_t chunk_offset,
                                  uint32_t data_len);
void encode_chunk_response(Bytes& out, uint8_t ext_id, uint32_t request_id, uint32_t chunk_offset,
                           const uint8_t* data, size_t n);
void encode_chunk_not_found(Bytes& out, uint8_t ext_id, uint32_t request_id, const uint8_t hash[32]);
void encode_chunk_error(Bytes& out, uint8_t ext_id, uint32_t request_id, uint32_t code, std::string_view msg);

// Decode the XET sub-payload (after ext_id).  Throws Error("UnexpectedEnd" | "UnknownXetType").
Message decode(ByteSpan data);

struct ExtCapabilities {
  int ut_xet_id = -1;    // 1..255 or -1
  int listen_port = -1;  // 1..65535 or -1
  std::string client;
};
std::string make_ext_handshake(uint16_t listen_port, uint8_t ut_xet_id = 1,
                               std::string_view client = kClientVersion);
ExtCapabilities parse_ext_handshake(ByteSpan payload);  // never throws: malformed -> empty caps

}  // namespace zest::bep_xet
