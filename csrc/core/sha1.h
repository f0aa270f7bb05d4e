// SHA-1 (FIPS 180-4) with an x86 SHA-NI fast path, and the zest peer identity helpers.
//
// Reference: src/peer_id.zig:1-63 — peer id "-ZE0200-" + 12 random bytes (:10-18) and
// info_hash = SHA1("zest-xet-v1:" || xorb_hash[32]) (:21-33), one BitTorrent swarm per xorb.
// Bench row `sha1_info_hash` (src/bench.zig:225-238).
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <string>

namespace zest {

using Sha1Digest = std::array<uint8_t, 20>;

class Sha1 {
 public:
  Sha1();
  void update(const void* data, size_t n);
  Sha1Digest finish();
  static Sha1Digest hash(const void* data, size_t n);
  static const char* backend();  // "sha-ni" or "portable"

 private:
  uint32_t h_[5];
  uint8_t buf_[64];
  size_t buf_len_ = 0;
  uint64_t total_ = 0;
};

namespace peer_id {
constexpr const char* kClientPrefix = "-ZE0402-";  // Azureus style: ZE = zest, 04.02
constexpr const char* kInfoHashPrefix = "zest-xet-v1:";
using PeerId = std::array<uint8_t, 20>;
PeerId generate();
// info_hash = SHA1("zest-xet-v1:" || xorb_hash), the BT swarm id of a xorb.
Sha1Digest info_hash(const uint8_t xorb_hash[32]);
}  // namespace peer_id

}  // namespace zest
