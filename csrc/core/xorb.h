// Xorb serialization: chunk headers, builder, reader/extractor and the XETBLOB footer.
//
// Reference: zig-xet `xorb` XorbReader.extractChunkRange (called at xet_bridge.zig:256-257 and
// parallel_download.zig:65-66); xorbs are capped at 64 MiB (bt_wire.zig:21-22).  Byte layout
// (8-byte chunk header; CasObjectInfoV1 footer "XETBLOB"/"XBLBHSH"/"XBLBBND") is pinned against
// xorbs produced by hf_xet in tests/test_xet_golden.py.
#pragma once

#include <optional>
#include <vector>

#include "common.h"
#include "lz4.h"
#include "xet_hash.h"

namespace zest::xet {

constexpr size_t kChunkHeaderLen = 8;
constexpr uint8_t kChunkHeaderVersion = 0;
constexpr size_t kMaxXorbBytes = 64ull << 20;
constexpr size_t kMaxXorbChunks = 8192;

struct ChunkHeader {
  uint8_t version = 0;
  uint32_t clen = 0;
  Scheme scheme = Scheme::None;
  uint32_t ulen = 0;
};
void write_chunk_header(uint8_t* p, const ChunkHeader& h);
ChunkHeader read_chunk_header(const uint8_t* p);  // throws Error("CorruptChunk")

// One chunk inside a serialized run (offsets relative to the run start).
struct ChunkEntry {
  uint64_t header_off;    // offset of the 8-byte header
  uint32_t clen;          // payload length
  Scheme scheme;
  uint32_t ulen;          // uncompressed length
  uint64_t unpacked_off;  // prefix sum of ulen
};

struct XorbFooter {
  Hash xorb_hash{};
  std::vector<Hash> chunk_hashes;
  std::vector<uint32_t> chunk_boundaries;   // serialized END offset of each chunk
  std::vector<uint32_t> unpacked_offsets;   // cumulative uncompressed END offset
};

// Walk chunk headers of a serialized run.  If the run carries a footer, the walk stops at it.
std::vector<ChunkEntry> index_chunks(const uint8_t* data, size_t n);
// Locate and parse a XETBLOB footer; returns nullopt when absent.  `footer_start` gets its offset.
std::optional<XorbFooter> parse_footer(const uint8_t* data, size_t n, size_t* footer_start = nullptr);
Bytes serialize_footer(const XorbFooter& f);

// Decompress chunks [start, end) (indices local to the run) and append to `out`.  If `hashes` is
// non-null, the chunk hashes of the extracted chunks are appended to it.
void extract_chunk_range(const uint8_t* data, size_t n, uint32_t start, uint32_t end, Bytes& out,
                         std::vector<HashSize>* hashes = nullptr);

// Verify a complete xorb: every chunk hash against the footer and the Merkle root against
// `expected` (or the footer's hash if expected is null).  Throws Error("HashMismatch").
void verify_xorb(const uint8_t* data, size_t n, const Hash* expected = nullptr);

class XorbBuilder {
 public:
  explicit XorbBuilder(CompressionPolicy policy = CompressionPolicy::Auto) : policy_(policy) {}
  bool fits(size_t ulen) const;
  // Append one chunk (hashes + compresses it).  Returns the chunk index inside the xorb.
  uint32_t add_chunk(const uint8_t* data, size_t n);
  // Append an already compressed chunk with a known hash.
  uint32_t add_compressed(const Hash& h, Scheme s, const uint8_t* payload, size_t clen, uint32_t ulen);
  size_t num_chunks() const { return hashes_.size(); }
  size_t serialized_size() const { return body_.size(); }
  uint64_t unpacked_size() const { return unpacked_; }
  Hash hash() const;  // Merkle root over chunk hashes
  const std::vector<Hash>& chunk_hashes() const { return hashes_; }
  const std::vector<uint32_t>& chunk_ulens() const { return ulens_; }
  const std::vector<uint32_t>& chunk_boundaries() const { return bounds_; }
  const Bytes& body() const { return body_; }
  // Full serialized xorb (body + footer).
  Bytes serialize(bool with_footer = true) const;
  void clear();

 private:
  CompressionPolicy policy_;
  Bytes body_;
  std::vector<Hash> hashes_;
  std::vector<uint32_t> ulens_;
  std::vector<uint32_t> bounds_;
  std::vector<uint32_t> unpacked_ends_;
  uint64_t unpacked_ = 0;
  Bytes scratch_;
};

}  // namespace zest::xet
