// Shared helpers for the zest host core: byte-order helpers, Status/Error, spans.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace zest {

using Bytes = std::vector<uint8_t>;

// Error type thrown by every native component. `code` is a short stable identifier that the
// Python layer and tests match on (e.g. "UnexpectedEnd", "LeadingZero", "HashMismatch").
class Error : public std::runtime_error {
 public:
  Error(std::string code, const std::string& msg = "")
      : std::runtime_error(msg.empty() ? code : code + ": " + msg), code_(std::move(code)) {}
  const std::string& code() const { return code_; }

 private:
  std::string code_;
};

struct ByteSpan {
  const uint8_t* data = nullptr;
  size_t size = 0;
  ByteSpan() = default;
  ByteSpan(const uint8_t* d, size_t n) : data(d), size(n) {}
  ByteSpan(const Bytes& b) : data(b.data()), size(b.size()) {}  // NOLINT
  ByteSpan(std::string_view s) : data(reinterpret_cast<const uint8_t*>(s.data())), size(s.size()) {}  // NOLINT
  std::string_view sv() const { return {reinterpret_cast<const char*>(data), size}; }
  ByteSpan sub(size_t off, size_t n) const { return {data + off, n}; }
};

inline uint32_t load_le32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t load_le64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
inline void store_le32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }
inline void store_le64(uint8_t* p, uint64_t v) { std::memcpy(p, &v, 8); }
inline uint32_t load_be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline uint16_t load_be16(const uint8_t* p) { return uint16_t((p[0] << 8) | p[1]); }
inline void store_be32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 24);
  p[1] = uint8_t(v >> 16);
  p[2] = uint8_t(v >> 8);
  p[3] = uint8_t(v);
}
inline void store_be16(uint8_t* p, uint16_t v) {
  p[0] = uint8_t(v >> 8);
  p[1] = uint8_t(v);
}
inline uint32_t load_le24(const uint8_t* p) { return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16); }
inline void store_le24(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v);
  p[1] = uint8_t(v >> 8);
  p[2] = uint8_t(v >> 16);
}

inline void append(Bytes& out, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  out.insert(out.end(), b, b + n);
}
inline void append(Bytes& out, std::string_view s) { append(out, s.data(), s.size()); }

}  // namespace zest
