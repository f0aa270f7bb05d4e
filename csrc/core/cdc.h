// GearHash content-defined chunking (Xet CDC: min 8 KiB / target 64 KiB / max 128 KiB).
//
// Reference: zig-xet `chunking` (CLAUDE.md:21; DESIGN.md:267-273).  Semantics pinned against
// hf_xet.hash_files() (tests/test_xet_golden.py): after each boundary the first
// (min - 64 - 1) bytes are skipped, the gear hash restarts from 0, and a boundary is declared
// after byte i when (h & mask) == 0, or when the chunk reaches the maximum size.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace zest::xet {

struct CdcParams {
  size_t target = 65536;
  size_t min_size = 65536 / 8;
  size_t max_size = 65536 * 2;
  uint64_t mask() const;  // (target-1) shifted to the top bits
};

// Streaming chunker.  feed() returns the chunk END offsets (absolute, in bytes since start)
// discovered in this call; finish() returns the final tail boundary (if any bytes remain).
class Chunker {
 public:
  explicit Chunker(CdcParams p = {});
  void feed(const uint8_t* data, size_t n, std::vector<uint64_t>& ends);
  void finish(std::vector<uint64_t>& ends);

 private:
  CdcParams p_;
  uint64_t mask_;
  uint64_t h_ = 0;
  uint64_t total_ = 0;      // bytes consumed so far
  uint64_t chunk_len_ = 0;  // bytes in the current chunk
};

// One-shot: chunk end offsets for a whole buffer.
std::vector<uint64_t> chunk_ends(const uint8_t* data, size_t n, CdcParams p = {});

// Gear hash of a full 64-byte window ending at data[i] (window = data[i-63..i]); the
// position-independent form used by the GPU candidate kernel.
uint64_t gear_window_hash(const uint8_t* data, size_t i);

}  // namespace zest::xet

namespace zest::xet {
// Apply the min/max chunk-size rule to sorted candidate END offsets (positions i+1 whose
// full-window gear hash matched) over a stream of n bytes -> chunk END offsets.  Used with the
// GPU candidate kernel (csrc/gpu/synth.hip); equivalent to Chunker over the same bytes.
std::vector<uint64_t> select_boundaries(const uint64_t* cand, size_t n_cand, uint64_t n, size_t min_size,
                                        size_t max_size);
}  // namespace zest::xet
