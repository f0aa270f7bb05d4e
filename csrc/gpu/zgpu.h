// Device-side descriptors and the C ABI of the zest HIP/CDNA4 kernel library (gfx950).
//
// Pipeline for one batch of fetched xorb ranges ("terms"):
//   zg_index_terms   one thread per term walks the 8-byte chunk headers -> ChunkDesc[]   (K4)
//   zg_place_chunks  one wave per chunk: scheme 0 -> aligned copy, LZ4/BG4 -> LDS decode (K3)
//   zg_hash_chunks   keyed BLAKE3 of the placed bytes -> chunk hashes (K1; lane per 1 KiB leaf)
//   zg_merkle_files  one workgroup per file: Xet Merkle tree -> root -> file hash compare (K2)
// plus zg_cdc_candidates (K5), zg_pack_xorbs (K7) and synthetic data generators.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// A fetched byte run holding whole chunks [chunk 0 .. n_chunks) of one xorb range.
typedef struct ZgTerm {
  uint64_t src;         // byte offset of the first chunk header in the src (staging) buffer
  uint64_t src_len;     // bytes in the run
  uint64_t dst;         // byte offset of the first chunk's output in the dst (arena) buffer
  uint32_t chunk_base;  // index of the first chunk in the ChunkDesc / hash arrays
  uint32_t n_chunks;    // chunks the run must contain
  uint64_t ulen;        // expected total uncompressed bytes (0 = don't check)
} ZgTerm;

typedef struct ZgChunk {
  uint64_t src;     // payload offset in src buffer (after the 8-byte header)
  uint64_t dst;     // output offset in dst buffer
  uint32_t clen;    // compressed payload length
  uint32_t ulen;    // uncompressed length
  uint32_t scheme;  // 0 none, 1 LZ4 frame, 2 BG4+LZ4 frame
  uint32_t term;    // owning term (for error reports)
} ZgChunk;

// One Merkle job: n leaves (hash[32] + size) -> root; optional expected file hash compare.
typedef struct ZgMerkleJob {
  uint64_t leaf_base;  // index of the first leaf in the hash/size arrays
  uint64_t n_leaves;
  uint32_t want_file_hash;  // 1: result = file hash (keyed zero-salt of root); 0: raw root
  uint32_t pad;
} ZgMerkleJob;

// Error word layout written by kernels (first error wins via atomicCAS):
//   code << 32 | index.  Codes:
enum {
  ZG_OK = 0,
  ZG_ERR_HEADER = 1,       // bad chunk header (version/scheme)
  ZG_ERR_RANGE = 2,        // chunk extends past its run
  ZG_ERR_COUNT = 3,        // run has a different chunk count / size than planned
  ZG_ERR_LZ4 = 4,          // malformed LZ4 frame / block
  ZG_ERR_SIZE = 5,         // decoded size != header ulen
  ZG_ERR_HASH = 6,         // hash mismatch
  ZG_ERR_CAPACITY = 7,     // chunk larger than kernel capacity
};

// All launchers return hipError_t of the launch and never synchronize.
hipError_t zg_index_terms(const uint8_t* src, const ZgTerm* terms, int n_terms, ZgChunk* chunks,
                          unsigned long long* err, hipStream_t stream);
// Descriptors are bounds-checked in-kernel against src_n / dst_n (bytes).  A clip window narrower
// than [0, dst_n) needs `clip_scratch` (ZG_CLIP_SCRATCH_BYTES of device memory owned by the caller,
// one per concurrently running launch): compressed chunks that straddle the window decode there
// before their clipped part is copied out.  Without it such a launch returns hipErrorInvalidValue.
#define ZG_CLIP_SCRATCH_BYTES (2u * (128u * 1024u + 256u))
// Unclipped launches decode LZ4 chunks with the batched decoder (lz4seq.hip: scalar parse into
// lane registers + lane-parallel execute); clipped ones with the LDS-ring decoder (ingest.hip).
// K4 parallel header walk: candidate scan over the span [0, src_n) of src + per-term sort/link in
// LDS; a term whose candidates are not exactly its chunk chain takes the serial walk (same records
// and errors as zg_index_terms).  Terms sorted by src.  scratch: zg_index_scratch_bytes(n_terms)
// of device memory, private to the stream (null / too small: zg_index_terms).
size_t zg_index_scratch_bytes(int n_terms);
hipError_t zg_index_terms_scan(const uint8_t* src, uint64_t src_n, const ZgTerm* terms, int n_terms, ZgChunk* chunks,
                               unsigned long long* err, uint8_t* scratch, size_t scratch_bytes, hipStream_t stream);
hipError_t zg_place_chunks(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                           const ZgChunk* chunks, int n_chunks, uint64_t clip_lo, uint64_t clip_hi,
                           uint8_t* clip_scratch, unsigned long long* err, hipStream_t stream);
hipError_t zg_lz4_batched_decode(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                 const ZgChunk* chunks, int n_chunks, unsigned long long* err, hipStream_t stream);
// Two-kernel decode (lane-per-chunk parse into records, wave-per-chunk execute) with a caller-owned
// scratch of zg_lz4_rec_scratch_bytes(n_chunks, src_n) bytes (one per concurrently running
// launch); a null or short scratch runs zg_lz4_batched_decode instead.
size_t zg_lz4_rec_scratch_bytes(int n_chunks, uint64_t src_n);
hipError_t zg_lz4_decode_records(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                 const ZgChunk* chunks, int n_chunks, unsigned long long* err, uint8_t* scratch,
                                 size_t scratch_bytes, hipStream_t stream);
// Producer/consumer decode: two waves per chunk (scalar parse -> LDS batch ring -> lane-parallel
// execute), for launches with fewer chunks than resident waves.  grid_cap: pairs (0 = 4096).
hipError_t zg_lz4_pair_decode(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                              int n_chunks, unsigned long long* err, int grid_cap, hipStream_t stream);
// Same with an explicit persistent-grid cap in blocks of 4 waves (0 = default 2048).
hipError_t zg_lz4_batched_decode_grid(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                      const ZgChunk* chunks, int n_chunks, unsigned long long* err, int grid_cap,
                                      hipStream_t stream);
// K1 keyed BLAKE3 of placed chunks (hashes[hash_index_base + c], sizes likewise when non-null) or of
// raw (offset, len) messages (key_mode 0 Xet data key, 1 node key, 2 plain, 3 zero key; a message
// over 128 KiB gets an all-ones hash).  With `scratch` (>= zg_hash_scratch_bytes(n, total message
// bytes) of device memory owned by the caller, one per concurrently running launch) the leaf-flat
// pipeline of blake3_flat.hip runs; without it, one wave per message (ingest.hip).
size_t zg_hash_scratch_bytes(int n, uint64_t total_bytes);
// Scratch of one zg_ingest_chunks launch (hash scratch + the decoder's BG4 staging, which share it).
size_t zg_ingest_scratch_bytes(int n, uint64_t total_bytes);
hipError_t zg_hash_chunks(const uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks, int n_chunks,
                          uint8_t* hashes, uint64_t* sizes, uint32_t hash_index_base, uint8_t* scratch,
                          size_t scratch_bytes, hipStream_t stream);
hipError_t zg_hash_ranges(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lens, int n,
                          uint8_t* hashes, int key_mode, uint8_t* scratch, size_t scratch_bytes, hipStream_t stream);
hipError_t zg_hash_chunks_flat(const uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks, int n_chunks,
                               uint8_t* hashes, uint64_t* sizes, uint8_t* scratch, size_t scratch_bytes,
                               hipStream_t stream);
hipError_t zg_hash_ranges_flat(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lens, int n,
                               uint8_t* hashes, int key_mode, uint8_t* scratch, size_t scratch_bytes,
                               hipStream_t stream);
// Fused K3a + K1: uncompressed chunks are copied src -> dst by the hashing waves themselves (and
// hashed from src); compressed ones must already be decoded into dst.  Descriptors out of bounds are
// not placed, hash over empty leaves (never their real hash) and set ZG_ERR_RANGE (chunk index) in `err` (may be null).
hipError_t zg_lz4_pair_decode_hash(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                   const ZgChunk* chunks, int n_chunks, unsigned long long* err, int grid_cap,
                                   uint8_t* hashes, uint64_t* sizes, hipStream_t stream);
// `stage` (>= zg_lz4_stage_bytes(n) of device memory, or null): BG4 chunks decode their grouped
// stream there and are written to dst once, whole lines at a time (ZG_BG4_STAGE=0 turns it off).
hipError_t zg_lz4_decode_ingest(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                                int n_chunks, unsigned long long* err, uint8_t* hashes, uint64_t* sizes, int* hashed,
                                uint8_t* stage, size_t stage_bytes, hipStream_t stream);
size_t zg_lz4_stage_bytes(int n_chunks);
hipError_t zg_lz4_pair_decode_hash_staged(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                          const ZgChunk* chunks, int n_chunks, unsigned long long* err, int grid_cap,
                                          uint8_t* hashes, uint64_t* sizes, uint8_t* stage, size_t stage_bytes,
                                          hipStream_t stream);
hipError_t zg_place_hash_flat_raw(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n,
                                  const ZgChunk* chunks, int n_chunks, unsigned long long* err, uint8_t* hashes,
                                  uint64_t* sizes, uint8_t* scratch, size_t scratch_bytes, hipStream_t stream);
hipError_t zg_place_hash_flat(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                              int n_chunks, unsigned long long* err, uint8_t* hashes, uint64_t* sizes, uint8_t* scratch,
                              size_t scratch_bytes, hipStream_t stream);
// One ingest launch sequence for an unclipped batch: LZ4/BG4 decode of the compressed chunks (only
// when `has_compressed`), then the fused place + hash (hashes[hash_index_base + c]).  Replaces
// zg_place_chunks + zg_hash_chunks (2 passes over the arena) with one pass; `scratch` is required.
hipError_t zg_ingest_chunks(const uint8_t* src, uint64_t src_n, uint8_t* dst, uint64_t dst_n, const ZgChunk* chunks,
                            int n_chunks, int has_compressed, unsigned long long* err, uint8_t* hashes,
                            uint64_t* sizes, uint32_t hash_index_base, uint8_t* scratch, size_t scratch_bytes,
                            hipStream_t stream);
hipError_t zg_merkle(const uint8_t* leaf_hashes, const uint64_t* leaf_sizes, const ZgMerkleJob* jobs,
                     int n_jobs, uint8_t* roots, uint8_t* scratch, uint64_t scratch_bytes,
                     hipStream_t stream);
size_t zg_merkle_scratch_bytes(uint64_t max_leaves_per_job, int n_jobs);
hipError_t zg_compare_hashes(const uint8_t* got, const uint8_t* want, int n, unsigned long long* err,
                             hipStream_t stream);
// CDC: candidate END offsets (i+1) where the full-window gear hash has (h & mask) == 0.
hipError_t zg_cdc_candidates(const uint8_t* data, uint64_t n, uint64_t mask, uint64_t* out,
                             unsigned long long* count, uint64_t capacity, hipStream_t stream);
// Synthetic content.  mode 0: uniform random bytes; mode 1: bf16 ~ N(0, 0.02).
hipError_t zg_fill_synthetic(uint8_t* dst, uint64_t n, uint64_t seed, uint64_t stream_offset, int mode,
                             hipStream_t stream);
// K7b: compress chunks (optional BG4 grouping into `scratch`, slot `in_slot` bytes per chunk) into
// LZ4 frames at out + c * out_slot; out_len[c] = frame bytes, or 0 when the chunk does not compress.
// hc64 / hc256: frame header checksum bytes for the 64 KiB / 256 KiB block-size descriptors.
hipError_t zg_compress_chunks(const uint8_t* data, const uint64_t* offs, const uint32_t* lens, int n, int bg4,
                              uint8_t* scratch, uint64_t in_slot, uint8_t* out, uint64_t out_slot, uint32_t* out_len,
                              uint32_t hc64, uint32_t hc256, hipStream_t stream);
// Serialize chunks (header + payload copied from per-chunk device addresses) into xorb bodies.
hipError_t zg_pack_frames(const uint64_t* src, const uint32_t* clen, const uint32_t* ulen, const uint8_t* scheme,
                          const uint64_t* out_off, int n, uint8_t* out, hipStream_t stream);

// Pack uncompressed chunks into serialized xorb bodies: header (version 0, scheme 0) + payload.
hipError_t zg_pack_chunks(const uint8_t* data, const uint64_t* data_off, const uint32_t* lens,
                          const uint64_t* out_off, int n, uint8_t* out, hipStream_t stream);

// K8: pull each segment's bytes from a peer's IPC-mapped arena (xGMI) into this GPU's arena;
// every segment is read concurrently.  src[i] and dst[i] must be congruent mod 16.
enum { kZgMaxPeerSegs = 16 };
typedef struct ZgPeerSegs {
  uint64_t src[kZgMaxPeerSegs];
  uint64_t dst[kZgMaxPeerSegs];
  uint64_t n[kZgMaxPeerSegs];
  int nseg;
} ZgPeerSegs;
hipError_t zg_peer_gather(const ZgPeerSegs* segs, hipStream_t stream);

int zg_device_count(void);
// K6: out[i] (20 B) = SHA1("zest-xet-v1:" || hashes[i] (32 B)); out must be 4-byte aligned.
hipError_t zg_sha1_info_hash(const uint8_t* hashes, int n, uint8_t* out, hipStream_t stream);

#ifdef __cplusplus
}
#endif
