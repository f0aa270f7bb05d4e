// Xet content addressing: chunk hashes, Merkle aggregation, xorb/file hashes, hex conventions.
//
// Reference call sites: zig-xet `hashing` (not vendored) used at xet_bridge.zig:154 and
// server.zig:203 (Xet hex = 4 little-endian u64 words, CONTRIBUTING.md:134-136) versus the
// reference's own byte-wise storage.zig:91-99 hashToHex.  Merkle rule per CONTRIBUTING.md:144-146
// (branching factor 4, domain-separation keys).  All constants are pinned by hf_xet golden vectors
// in tests/test_xet_golden.py.
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace zest::xet {

using Hash = std::array<uint8_t, 32>;

extern const uint8_t kDataKey[32];          // chunk hash key
extern const uint8_t kInternalNodeKey[32];  // Merkle internal node key
constexpr uint64_t kMeanBranching = 4;
constexpr size_t kMaxChildren = 2 * kMeanBranching + 1;  // 9

// "Xet hex": the 32 bytes as 4 little-endian u64 words, each printed %016x.
std::string to_hex(const Hash& h);
Hash from_hex(std::string_view hex);  // throws Error("InvalidHash")
// Plain byte-wise lowercase hex (storage.zig:91-99 convention; used by legacy chunk cache).
std::string to_bytewise_hex(const uint8_t* p, size_t n);
Bytes from_bytewise_hex(std::string_view hex);

Hash chunk_hash(const uint8_t* data, size_t len);
Hash internal_node_hash(const uint8_t* data, size_t len);

struct HashSize {
  Hash hash;
  uint64_t size;
};

// Cut point for the next Merkle group starting at `nodes[0]` (returns #children in the group).
size_t next_merge_cut(const HashSize* nodes, size_t n);
// Hash of one group: keyed BLAKE3 over lines "{xet_hex} : {size}\n".
HashSize merge_group(const HashSize* nodes, size_t n);
// Full aggregated Merkle root (xorb hash when fed the xorb's chunks).
Hash merkle_root(const std::vector<HashSize>& leaves);
// File hash = BLAKE3 keyed with a 32-byte salt (all-zero by default) of the Merkle root.
Hash file_hash(const std::vector<HashSize>& chunks);
Hash file_hash_from_root(const Hash& root, bool empty);

}  // namespace zest::xet
