#include "xet_hash.h"

#include <cstdio>
#include <cstring>

#include "blake3.h"

namespace zest::xet {

const uint8_t kDataKey[32] = {102, 151, 245, 119, 91,  149, 80,  222, 49,  53,  203,
                              172, 165, 151, 24,  28,  157, 228, 33,  16,  155, 235,
                              43,  88,  180, 208, 176, 75,  147, 173, 242, 41};
const uint8_t kInternalNodeKey[32] = {1,   126, 197, 199, 165, 71,  41,  150, 253, 148, 102,
                                      102, 180, 138, 2,   230, 93,  221, 83,  111, 55,  199,
                                      109, 210, 248, 99,  82,  230, 74,  83,  113, 63};

namespace {
const char kHexDigits[] = "0123456789abcdef";
int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
}  // namespace

std::string to_hex(const Hash& h) {
  std::string s(64, '0');
  for (int w = 0; w < 4; ++w) {
    uint64_t v = load_le64(h.data() + 8 * w);
    for (int d = 15; d >= 0; --d) {
      s[16 * w + d] = kHexDigits[v & 15];
      v >>= 4;
    }
  }
  return s;
}

Hash from_hex(std::string_view hex) {
  if (hex.size() != 64) throw Error("InvalidHash", "expected 64 hex chars");
  Hash h{};
  for (int w = 0; w < 4; ++w) {
    uint64_t v = 0;
    for (int d = 0; d < 16; ++d) {
      int x = hexval(hex[16 * w + d]);
      if (x < 0) throw Error("InvalidHash", "non-hex character");
      v = (v << 4) | uint64_t(x);
    }
    store_le64(h.data() + 8 * w, v);
  }
  return h;
}

std::string to_bytewise_hex(const uint8_t* p, size_t n) {
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = kHexDigits[p[i] >> 4];
    s[2 * i + 1] = kHexDigits[p[i] & 15];
  }
  return s;
}

Bytes from_bytewise_hex(std::string_view hex) {
  if (hex.size() % 2) throw Error("InvalidHash", "odd hex length");
  Bytes out(hex.size() / 2);
  for (size_t i = 0; i < out.size(); ++i) {
    int a = hexval(hex[2 * i]), b = hexval(hex[2 * i + 1]);
    if (a < 0 || b < 0) throw Error("InvalidHash", "non-hex character");
    out[i] = uint8_t(a * 16 + b);
  }
  return out;
}

Hash chunk_hash(const uint8_t* data, size_t len) {
  Hash h;
  blake3::keyed_hash(kDataKey, data, len, h.data());
  return h;
}

Hash internal_node_hash(const uint8_t* data, size_t len) {
  Hash h;
  blake3::keyed_hash(kInternalNodeKey, data, len, h.data());
  return h;
}

size_t next_merge_cut(const HashSize* nodes, size_t n) {
  if (n <= 2) return n;
  const size_t end = std::min(kMaxChildren, n);
  for (size_t i = 2; i < end; ++i) {
    const uint64_t w3 = load_le64(nodes[i].hash.data() + 24);
    if (w3 % kMeanBranching == 0) return i + 1;
  }
  return end;
}

HashSize merge_group(const HashSize* nodes, size_t n) {
  char buf[kMaxChildren * 96];
  size_t pos = 0;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    std::string hx = to_hex(nodes[i].hash);
    std::memcpy(buf + pos, hx.data(), 64);
    pos += 64;
    pos += std::snprintf(buf + pos, sizeof(buf) - pos, " : %llu\n",
                         static_cast<unsigned long long>(nodes[i].size));
    total += nodes[i].size;
  }
  return {internal_node_hash(reinterpret_cast<const uint8_t*>(buf), pos), total};
}

Hash merkle_root(const std::vector<HashSize>& leaves) {
  if (leaves.empty()) return Hash{};
  std::vector<HashSize> hv = leaves;
  while (hv.size() > 1) {
    size_t w = 0, r = 0;
    while (r < hv.size()) {
      size_t cut = next_merge_cut(hv.data() + r, hv.size() - r);
      hv[w++] = merge_group(hv.data() + r, cut);
      r += cut;
    }
    hv.resize(w);
  }
  return hv[0].hash;
}

Hash file_hash_from_root(const Hash& root, bool empty) {
  if (empty) return Hash{};
  static const uint8_t zero_key[32] = {0};
  Hash h;
  blake3::keyed_hash(zero_key, root.data(), 32, h.data());
  return h;
}

Hash file_hash(const std::vector<HashSize>& chunks) {
  return file_hash_from_root(merkle_root(chunks), chunks.empty());
}

}  // namespace zest::xet
