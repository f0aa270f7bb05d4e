// LZ4 block + frame codec, xxHash32, and Xet's ByteGrouping4 (BG4) transform.
//
// Xet chunk payloads use the LZ4 *frame* format (magic 04 22 4D 18, independent blocks, no
// checksums; block-max 64 KB for payloads <= 64 KiB, else 256 KB) — pinned against xorbs written
// by hf_xet in tests/test_xet_golden.py.  The reference reaches this through zig-xet's
// `compression` module via XorbReader.extractChunkRange (xet_bridge.zig:256-257,
// parallel_download.zig:65-66).  This host codec is the CPU oracle for csrc/gpu/lz4_kernels.hip.
#pragma once

#include <cstddef>
#include <cstdint>

#include "common.h"

namespace zest::lz4 {

uint32_t xxh32(const void* data, size_t len, uint32_t seed);

// Worst-case compressed size of a block.
size_t block_bound(size_t n);
// Compress one block (greedy hash-chain-free matcher).  Returns compressed size.
size_t compress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t cap);
// Decompress a block into dst[dst_pos .. dst_cap); matches may reference dst[0 .. dst_pos)
// (dependent-block prefix).  Returns bytes produced; throws Error("CorruptLz4") on malformed input.
// Decodes into dst[dst_pos, ...) and returns the bytes produced.  May write scratch bytes past the
// produced output, anywhere below dst_cap: pass the end of the region this block's output owns.
size_t decompress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_pos, size_t dst_cap);

// Frame format.
constexpr uint32_t kFrameMagic = 0x184D2204u;
Bytes compress_frame(const uint8_t* src, size_t n);
// Decompress a whole frame; `expected` (if non-zero) pre-sizes / validates the output.
Bytes decompress_frame(const uint8_t* src, size_t n, size_t expected = 0);
// Decompress into a caller buffer of exactly `out_len` bytes (the chunk header's ulen).
void decompress_frame_into(const uint8_t* src, size_t n, uint8_t* out, size_t out_len);

}  // namespace zest::lz4

namespace zest::bg4 {
// Split bytes into 4 groups (i % 4) laid out back to back; join is the inverse.
void split(const uint8_t* src, size_t n, uint8_t* dst);
void join(const uint8_t* src, size_t n, uint8_t* dst);
}  // namespace zest::bg4

namespace zest::xet {

enum class Scheme : uint8_t { None = 0, LZ4 = 1, BG4LZ4 = 2 };
enum class CompressionPolicy { None, LZ4, BG4, Auto };

// Compress one chunk payload; returns the scheme actually used (None if no gain).
Scheme compress_chunk(const uint8_t* data, size_t n, CompressionPolicy policy, Bytes& out);
// Decompress a chunk payload into out[0..ulen).
void decompress_chunk(Scheme s, const uint8_t* payload, size_t clen, uint8_t* out, size_t ulen);

}  // namespace zest::xet
