// BLAKE3 (https://github.com/BLAKE3-team/BLAKE3-specs) — host implementation.
//
// Portable compression plus AVX2 (8-way) and AVX-512 (16-way) "hash many" paths that hash
// independent 1 KiB chunks / parent blocks in SIMD lanes, chosen at runtime by CPU feature
// detection.  This is the CPU oracle for the HIP kernels in csrc/gpu/blake3_dev.h and the
// backend of `zest bench --synthetic` row `blake3_64kb` (reference: src/bench.zig:207-223,
// which hashes 64 KiB of 0x42 with Zig's std BLAKE3).
#pragma once

#include <cstddef>
#include <cstdint>

namespace zest::blake3 {

constexpr size_t kOutLen = 32;
constexpr size_t kKeyLen = 32;
constexpr size_t kBlockLen = 64;
constexpr size_t kChunkLen = 1024;

enum Flags : uint8_t {
  CHUNK_START = 1,
  CHUNK_END = 2,
  PARENT = 4,
  ROOT = 8,
  KEYED_HASH = 16,
  DERIVE_KEY_CONTEXT = 32,
  DERIVE_KEY_MATERIAL = 64,
};

extern const uint32_t kIV[8];

// One BLAKE3 compression; cv is updated in place with the first 8 output words.
void compress_in_place(uint32_t cv[8], const uint8_t block[64], uint8_t block_len, uint64_t counter,
                       uint8_t flags);

// Hash `n` independent inputs, each exactly `blocks` * 64 bytes, writing 32-byte CVs.
// The counter for input i is counter + (increment_counter ? i : 0).  `flags_start` is OR-ed into the
// first block and `flags_end` into the last block of every input.
void hash_many(const uint8_t* const* inputs, size_t n, size_t blocks, const uint32_t key[8],
               uint64_t counter, bool increment_counter, uint8_t flags, uint8_t flags_start,
               uint8_t flags_end, uint8_t* out);

// One-shot hashes.
void hash(const void* data, size_t len, uint8_t out[32]);
void keyed_hash(const uint8_t key[32], const void* data, size_t len, uint8_t out[32]);
// Generic: `key` words are the initial CV, `flags` the mode flag (0 or KEYED_HASH).
void hash_with_key(const uint32_t key[8], uint8_t flags, const void* data, size_t len, uint8_t out[32]);

// Name of the SIMD backend selected at runtime: "avx512", "avx2" or "portable".
const char* simd_backend();
// Force a backend (tests): "avx512" | "avx2" | "portable"; returns false if unsupported.
bool force_backend(const char* name);

}  // namespace zest::blake3
