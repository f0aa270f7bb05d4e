#include "bt_wire.h"

#include <cstring>

#include "bencode.h"

namespace zest::bt {

bool known_msg_id(uint8_t id) { return id <= kCancel || id == kExtended; }

void write_handshake(Bytes& out, const Sha1Digest& info_hash, const peer_id::PeerId& pid) {
  const size_t o = out.size();
  out.resize(o + kHandshakeLen);
  uint8_t* p = out.data() + o;
  p[0] = uint8_t(kProtocol.size());
  std::memcpy(p + 1, kProtocol.data(), kProtocol.size());
  std::memcpy(p + 20, kReserved, 8);
  std::memcpy(p + 28, info_hash.data(), 20);
  std::memcpy(p + 48, pid.data(), 20);
}

Handshake parse_handshake(const uint8_t* p) {
  if (p[0] != kProtocol.size() || std::memcmp(p + 1, kProtocol.data(), kProtocol.size()) != 0)
    throw Error("InvalidProtocolString");
  Handshake h;
  std::memcpy(h.reserved.data(), p + 20, 8);
  std::memcpy(h.info_hash.data(), p + 28, 20);
  std::memcpy(h.peer_id.data(), p + 48, 20);
  return h;
}

void write_message(Bytes& out, uint8_t id, const uint8_t* payload, size_t n) {
  const size_t o = out.size();
  out.resize(o + 5 + n);
  store_be32(out.data() + o, uint32_t(1 + n));
  out[o + 4] = id;
  if (n) std::memcpy(out.data() + o + 5, payload, n);
}

void write_keepalive(Bytes& out) { out.insert(out.end(), 4, 0); }

void write_extended(Bytes& out, uint8_t ext_id, const uint8_t* payload, size_t n) {
  const size_t o = out.size();
  out.resize(o + 6 + n);
  store_be32(out.data() + o, uint32_t(2 + n));
  out[o + 4] = kExtended;
  out[o + 5] = ext_id;
  if (n) std::memcpy(out.data() + o + 6, payload, n);
}

size_t frame_length(const uint8_t* p, size_t n) {
  if (n < 4) return 0;
  const uint32_t len = load_be32(p);
  if (len > kMaxMessage) throw Error("InvalidMessageSize");
  return 4 + size_t(len);
}

size_t parse_message(const uint8_t* p, size_t n, Message& m) {
  const size_t total = frame_length(p, n);
  if (total == 0 || n < total) return 0;
  const uint32_t len = uint32_t(total - 4);
  if (len == 0) {
    m.keepalive = true;
    m.id = 0;
    m.payload = {};
    return 4;
  }
  m.keepalive = false;
  m.id = p[4];
  if (!known_msg_id(m.id)) throw Error("InvalidMessageId", std::to_string(m.id));
  m.payload = ByteSpan(p + 5, len - 1);
  return total;
}

Extended parse_extended(ByteSpan payload) {
  if (payload.size < 1) throw Error("UnexpectedEnd");
  return {payload.data[0], payload.sub(1, payload.size - 1)};
}

}  // namespace zest::bt

namespace zest::bep_xet {

namespace {
void ext_header(Bytes& out, uint8_t ext_id, size_t xet_len) {
  const size_t o = out.size();
  out.resize(o + 6);
  store_be32(out.data() + o, uint32_t(2 + xet_len));
  out[o + 4] = bt::kExtended;
  out[o + 5] = ext_id;
}
void put_be32(Bytes& out, uint32_t v) {
  uint8_t b[4];
  store_be32(b, v);
  out.insert(out.end(), b, b + 4);
}
}  // namespace

void encode_chunk_request(Bytes& out, uint8_t ext_id, uint32_t request_id, const uint8_t hash[32],
                          uint32_t range_start, uint32_t range_end) {
  ext_header(out, ext_id, 45);
  out.push_back(kChunkRequest);
  put_be32(out, request_id);
  out.insert(out.end(), hash, hash + 32);
  put_be32(out, range_start);
  put_be32(out, range_end);
}

void encode_chunk_response_header(Bytes& out, uint8_t ext_id, uint32_t request_id, uint32_t chunk_offset,
                                  uint32_t data_len) {
  ext_header(out, ext_id, 13 + size_t(data_len));
  out.push_back(kChunkResponse);
  put_be32(out, request_id);
  put_be32(out, chunk_offset);
  put_be32(out, data_len);
}

void encode_chunk_response(Bytes& out, uint8_t ext_id, uint32_t request_id, uint32_t chunk_offset,
                           const uint8_t* data, size_t n) {
  encode_chunk_response_header(out, ext_id, request_id, chunk_offset, uint32_t(n));
  out.insert(out.end(), data, data + n);
}

void encode_chunk_not_found(Bytes& out, uint8_t ext_id, uint32_t request_id, const uint8_t hash[32]) {
  ext_header(out, ext_id, 37);
  out.push_back(kChunkNotFound);
  put_be32(out, request_id);
  out.insert(out.end(), hash, hash + 32);
}

void encode_chunk_error(Bytes& out, uint8_t ext_id, uint32_t request_id, uint32_t code, std::string_view msg) {
  ext_header(out, ext_id, 9 + msg.size());
  out.push_back(kChunkError);
  put_be32(out, request_id);
  put_be32(out, code);
  out.insert(out.end(), msg.begin(), msg.end());
}

Message decode(ByteSpan d) {
  if (d.size < 1) throw Error("UnexpectedEnd");
  Message m;
  const uint8_t t = d.data[0];
  const uint8_t* r = d.data + 1;
  const size_t n = d.size - 1;
  switch (t) {
    case kChunkRequest:
      if (n < 44) throw Error("UnexpectedEnd");
      m.type = kChunkRequest;
      m.request_id = load_be32(r);
      std::memcpy(m.hash.data(), r + 4, 32);
      m.range_start = load_be32(r + 36);
      m.range_end = load_be32(r + 40);
      return m;
    case kChunkResponse: {
      if (n < 12) throw Error("UnexpectedEnd");
      m.type = kChunkResponse;
      m.request_id = load_be32(r);
      m.chunk_offset = load_be32(r + 4);
      const uint32_t len = load_be32(r + 8);
      if (n - 12 < len) throw Error("UnexpectedEnd");
      m.data = ByteSpan(r + 12, len);
      return m;
    }
    case kChunkNotFound:
      if (n < 36) throw Error("UnexpectedEnd");
      m.type = kChunkNotFound;
      m.request_id = load_be32(r);
      std::memcpy(m.hash.data(), r + 4, 32);
      return m;
    case kChunkError:
      if (n < 8) throw Error("UnexpectedEnd");
      m.type = kChunkError;
      m.request_id = load_be32(r);
      m.error_code = load_be32(r + 4);
      m.data = ByteSpan(r + 8, n - 8);
      return m;
    default:
      throw Error("UnknownXetType", std::to_string(t));
  }
}

std::string make_ext_handshake(uint16_t listen_port, uint8_t ut_xet_id, std::string_view client) {
  std::string out;
  bencode::Encoder e(out);
  e.begin_dict();
  e.key("m").begin_dict().key(kExtName).integer(ut_xet_id).end();
  e.key("p").integer(listen_port);
  e.key("v").str(client);
  e.end();
  return out;
}

ExtCapabilities parse_ext_handshake(ByteSpan payload) {
  ExtCapabilities caps;
  try {
    bencode::Document doc;
    doc.parse(payload.sv());
    bencode::Ref root = doc.root();
    if (!root.is_dict()) return caps;
    bencode::Ref m = root.get("m");
    if (m.is_dict()) {
      int64_t id = m.get_int(kExtName, -1);
      if (id >= 1 && id <= 255) caps.ut_xet_id = int(id);
    }
    int64_t p = root.get_int("p", -1);
    if (p >= 1 && p <= 65535) caps.listen_port = int(p);
    caps.client = std::string(root.get_str("v"));
  } catch (const Error&) {
  }
  return caps;
}

}  // namespace zest::bep_xet
