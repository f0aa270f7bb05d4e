#include "lz4.h"

#include <algorithm>
#include <cstring>

#include <emmintrin.h>

namespace zest::lz4 {

namespace {
constexpr uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu, P5 = 0x165667B1u;
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t read32(const uint8_t* p) { return load_le32(p); }
inline uint64_t read64(const uint8_t* p) { return load_le64(p); }

constexpr size_t kMinMatch = 4;
constexpr size_t kMfLimit = 12;
constexpr size_t kLastLiterals = 5;
constexpr uint32_t kMaxOffset = 65535;
constexpr int kHashLog = 14;

inline uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

inline uint8_t* write_len(uint8_t* op, size_t len) {
  while (len >= 255) {
    *op++ = 255;
    len -= 255;
  }
  *op++ = uint8_t(len);
  return op;
}
}  // namespace

uint32_t xxh32(const void* vdata, size_t len, uint32_t seed) {
  const uint8_t* p = static_cast<const uint8_t*>(vdata);
  const uint8_t* end = p + len;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* limit = end - 16;
    do {
      v1 = rotl32(v1 + read32(p) * P2, 13) * P1;
      v2 = rotl32(v2 + read32(p + 4) * P2, 13) * P1;
      v3 = rotl32(v3 + read32(p + 8) * P2, 13) * P1;
      v4 = rotl32(v4 + read32(p + 12) * P2, 13) * P1;
      p += 16;
    } while (p <= limit);
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + P5;
  }
  h += uint32_t(len);
  while (p + 4 <= end) {
    h += read32(p) * P3;
    h = rotl32(h, 17) * P4;
    p += 4;
  }
  while (p < end) {
    h += (*p++) * P5;
    h = rotl32(h, 11) * P1;
  }
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

size_t block_bound(size_t n) { return n + n / 255 + 16; }

size_t compress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  if (cap < block_bound(n)) throw Error("Lz4BufferTooSmall");
  // Table holds positions from earlier calls too: every candidate is validated (range + bytes),
  // so stale entries are harmless and no per-call clear is needed.
  thread_local uint32_t table[1u << kHashLog];
  uint8_t* op = dst;
  size_t anchor = 0;
  if (n >= kMfLimit + 1) {
    const size_t mflimit = n - kMfLimit;
    const size_t matchlimit = n - kLastLiterals;
    size_t ip = 0;
    table[hash4(read32(src))] = 0;
    ip = 1;
    while (ip <= mflimit) {
      // Find a match with LZ4's skip acceleration.
      size_t cand = 0;
      bool found = false;
      unsigned attempts = 1u << 6;
      while (ip <= mflimit) {
        const uint32_t seq = read32(src + ip);
        const uint32_t h = hash4(seq);
        cand = table[h];
        table[h] = uint32_t(ip);
        if (cand < ip && ip - cand <= kMaxOffset && read32(src + cand) == seq) {
          found = true;
          break;
        }
        ip += (attempts++ >> 6);
      }
      if (!found) break;
      // Extend backwards.
      while (ip > anchor && cand > 0 && src[ip - 1] == src[cand - 1]) {
        --ip;
        --cand;
      }
      // Extend forwards.
      size_t len = kMinMatch;
      while (ip + len + 8 <= matchlimit) {
        uint64_t diff = read64(src + ip + len) ^ read64(src + cand + len);
        if (diff) {
          len += size_t(__builtin_ctzll(diff) >> 3);
          goto done;
        }
        len += 8;
      }
      while (ip + len < matchlimit && src[ip + len] == src[cand + len]) ++len;
    done:
      {
        const size_t lit = ip - anchor;
        uint8_t* token = op++;
        if (lit >= 15) {
          *token = 15 << 4;
          op = write_len(op, lit - 15);
        } else {
          *token = uint8_t(lit << 4);
        }
        std::memcpy(op, src + anchor, lit);
        op += lit;
        const uint32_t off = uint32_t(ip - cand);
        *op++ = uint8_t(off);
        *op++ = uint8_t(off >> 8);
        const size_t ml = len - kMinMatch;
        if (ml >= 15) {
          *token |= 15;
          op = write_len(op, ml - 15);
        } else {
          *token |= uint8_t(ml);
        }
      }
      ip += len;
      anchor = ip;
      if (ip <= mflimit) table[hash4(read32(src + ip - 2))] = uint32_t(ip - 2);
    }
  }
  // Last literals.
  const size_t lit = n - anchor;
  uint8_t* token = op++;
  if (lit >= 15) {
    *token = 15 << 4;
    op = write_len(op, lit - 15);
  } else {
    *token = uint8_t(lit << 4);
  }
  std::memcpy(op, src + anchor, lit);
  op += lit;
  return size_t(op - dst);
}

namespace {
inline void copy8(uint8_t* d, const uint8_t* s) { std::memcpy(d, s, 8); }
inline void copy16(uint8_t* d, const uint8_t* s) { std::memcpy(d, s, 16); }
}  // namespace

// Sequences are parsed one at a time (the format is serial), but copies take fast paths whenever the
// buffers have slack: literals of up to 16 bytes move as one 16-byte copy, matches whose source is at
// least 16 (8) bytes back move in 16 (8)-byte steps that may run past the match end.  Reads stay in
// [src, src + n) and in the output already written ([dst, dst + op)); writes stay below dst_cap and
// the bytes written past a sequence's end are overwritten by the following output.  BG4 planes of
// bf16 weights are exponent bytes with many short matches: per-sequence memcpy calls held the host
// decoder to ~0.6 GB/s per thread.
size_t decompress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_pos, size_t dst_cap) {
  size_t ip = 0, op = dst_pos;
  while (true) {
    // Fast loop: with >= 32 input bytes and >= 64 output bytes of slack, a sequence whose lengths fit
    // their token nibbles (literals <= 14, match <= 18: nearly every sequence of a BG4 exponent plane)
    // needs no length bytes and no bound checks but the offset's.  Its literals (read from
    // src[ip + 1, ip + 17) < n) and its match (written below op + 14 + 24 < dst_cap) move as fixed
    // 16 / 8-byte copies.  It cannot be the block's last sequence: after its literals >= 17 input
    // bytes remain.
    while (n - ip >= 32 && dst_cap - op >= 64) {
      const uint8_t token = src[ip];
      const size_t lit = token >> 4, ml = (token & 15) + kMinMatch;
      if (lit == 15 || ml == 15 + kMinMatch) break;  // length bytes follow: the general path
      copy16(dst + op, src + ip + 1);
      ip += 1 + lit;
      op += lit;
      const size_t off = size_t(src[ip]) | (size_t(src[ip + 1]) << 8);
      ip += 2;
      if (off == 0 || off > op) throw Error("CorruptLz4", "bad offset");
      uint8_t* d = dst + op;
      const uint8_t* s = d - off;  // >= dst
      if (off >= 16) {
        copy16(d, s);
        if (ml > 16) copy16(d + 16, s + 16);
      } else if (off >= 8) {
        copy8(d, s);
        copy8(d + 8, s + 8);
        if (ml > 16) copy8(d + 16, s + 16);
      } else {
        for (size_t i = 0; i < ml; ++i) d[i] = s[i];
      }
      op += ml;
    }
    if (ip >= n) throw Error("CorruptLz4", "truncated token");
    const uint8_t token = src[ip++];
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= n) throw Error("CorruptLz4", "truncated literal length");
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - ip || lit > dst_cap - op) throw Error("CorruptLz4", "literal overflow");
    if (lit <= 16 && n - ip >= 16 && dst_cap - op >= 16) {
      copy16(dst + op, src + ip);  // reads src[ip, ip + 16) < n; writes dst[op, op + 16) < dst_cap
    } else {
      std::memcpy(dst + op, src + ip, lit);
    }
    ip += lit;
    op += lit;
    if (ip == n) break;  // last sequence carries literals only
    if (n - ip < 2) throw Error("CorruptLz4", "truncated offset");
    const size_t off = size_t(src[ip]) | (size_t(src[ip + 1]) << 8);
    ip += 2;
    if (off == 0 || off > op) throw Error("CorruptLz4", "bad offset");
    size_t ml = token & 15;
    if (ml == 15) {
      uint8_t b;
      do {
        if (ip >= n) throw Error("CorruptLz4", "truncated match length");
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    ml += kMinMatch;
    if (ml > dst_cap - op) throw Error("CorruptLz4", "match overflow");
    uint8_t* d = dst + op;
    const uint8_t* s = d - off;         // >= dst: off <= op was checked above
    const size_t slack = dst_cap - op;  // >= ml
    if (off >= 16 && slack >= ml + 15) {
      // each 16-byte step reads [s + k, s + k + 16), entirely before d + k (off >= 16): written bytes
      for (size_t k = 0; k < ml; k += 16) copy16(d + k, s + k);
    } else if (off >= 8 && slack >= ml + 7) {
      for (size_t k = 0; k < ml; k += 8) copy8(d + k, s + k);
    } else if (off >= ml) {
      std::memcpy(d, s, ml);
    } else {
      for (size_t i = 0; i < ml; ++i) d[i] = s[i];  // overlapping short-offset match, byte by byte
    }
    op += ml;
  }
  return op - dst_pos;
}

Bytes compress_frame(const uint8_t* src, size_t n) {
  const bool small = n <= 65536;
  const size_t block_max = small ? 65536 : 262144;
  Bytes out;
  out.reserve(n + n / 255 + 64);
  uint8_t hdr[7];
  store_le32(hdr, kFrameMagic);
  hdr[4] = 0x60;                  // version 01, independent blocks, no checksums, no size
  hdr[5] = small ? 0x40 : 0x50;   // block max size 64 KB / 256 KB
  hdr[6] = uint8_t((xxh32(hdr + 4, 2, 0) >> 8) & 0xFF);
  append(out, hdr, 7);
  Bytes tmp(block_bound(block_max));
  for (size_t off = 0; off < n; off += block_max) {
    const size_t len = std::min(block_max, n - off);
    const size_t c = compress_block(src + off, len, tmp.data(), tmp.size());
    uint8_t sz[4];
    if (c >= len) {
      store_le32(sz, uint32_t(len) | 0x80000000u);
      append(out, sz, 4);
      append(out, src + off, len);
    } else {
      store_le32(sz, uint32_t(c));
      append(out, sz, 4);
      append(out, tmp.data(), c);
    }
  }
  uint8_t end[4] = {0, 0, 0, 0};
  append(out, end, 4);
  return out;
}

namespace {
struct FrameHeader {
  size_t header_len;
  bool block_checksum;
  bool content_checksum;
  bool independent;
  size_t block_max;
};

FrameHeader parse_header(const uint8_t* src, size_t n) {
  if (n < 7 || load_le32(src) != kFrameMagic) throw Error("CorruptLz4", "bad frame magic");
  const uint8_t flg = src[4], bd = src[5];
  if ((flg >> 6) != 1) throw Error("CorruptLz4", "unsupported frame version");
  FrameHeader h;
  h.independent = flg & 0x20;
  h.block_checksum = flg & 0x10;
  const bool has_size = flg & 0x08;
  h.content_checksum = flg & 0x04;
  const bool has_dict = flg & 0x01;
  const int bsid = (bd >> 4) & 7;
  if (bsid < 4) throw Error("CorruptLz4", "bad block size id");
  h.block_max = size_t(1) << (8 + 2 * bsid);
  size_t pos = 6 + (has_size ? 8 : 0) + (has_dict ? 4 : 0);
  if (n < pos + 1) throw Error("CorruptLz4", "truncated frame header");
  const uint8_t hc = uint8_t((xxh32(src + 4, pos - 4, 0) >> 8) & 0xFF);
  if (hc != src[pos]) throw Error("CorruptLz4", "header checksum mismatch");
  h.header_len = pos + 1;
  return h;
}
}  // namespace

void decompress_frame_into(const uint8_t* src, size_t n, uint8_t* out, size_t out_len) {
  FrameHeader h = parse_header(src, n);
  size_t ip = h.header_len, op = 0;
  while (true) {
    if (n - ip < 4) throw Error("CorruptLz4", "truncated block size");
    const uint32_t bs = load_le32(src + ip);
    ip += 4;
    if (bs == 0) break;
    const bool raw = bs & 0x80000000u;
    const size_t len = bs & 0x7FFFFFFFu;
    if (len > n - ip) throw Error("CorruptLz4", "truncated block");
    if (raw) {
      if (len > out_len - op) throw Error("CorruptLz4", "raw block overflow");
      std::memcpy(out + op, src + ip, len);
      op += len;
    } else {
      // Dependent blocks may reference earlier output: the whole buffer is the prefix.
      op += decompress_block(src + ip, len, out, op, out_len);
    }
    ip += len;
    if (h.block_checksum) ip += 4;
  }
  if (op != out_len) throw Error("CorruptLz4", "decompressed size mismatch");
}

Bytes decompress_frame(const uint8_t* src, size_t n, size_t expected) {
  if (expected) {
    Bytes out(expected);
    decompress_frame_into(src, n, out.data(), expected);
    return out;
  }
  // Unknown size: grow by decoding block by block.
  FrameHeader h = parse_header(src, n);
  Bytes out;
  size_t ip = h.header_len;
  while (true) {
    if (n - ip < 4) throw Error("CorruptLz4", "truncated block size");
    const uint32_t bs = load_le32(src + ip);
    ip += 4;
    if (bs == 0) break;
    const bool raw = bs & 0x80000000u;
    const size_t len = bs & 0x7FFFFFFFu;
    if (len > n - ip) throw Error("CorruptLz4", "truncated block");
    const size_t op = out.size();
    if (raw) {
      out.insert(out.end(), src + ip, src + ip + len);
    } else {
      out.resize(op + h.block_max);
      size_t got = decompress_block(src + ip, len, out.data(), op, op + h.block_max);
      out.resize(op + got);
    }
    ip += len;
    if (h.block_checksum) ip += 4;
  }
  return out;
}

}  // namespace zest::lz4

namespace zest::bg4 {

void split(const uint8_t* src, size_t n, uint8_t* dst) {
  const size_t q = n / 4, r = n % 4;
  size_t off[4];
  off[0] = 0;
  for (int g = 1; g < 4; ++g) off[g] = off[g - 1] + q + (size_t(g - 1) < r ? 1 : 0);
  uint8_t* d0 = dst + off[0];
  uint8_t* d1 = dst + off[1];
  uint8_t* d2 = dst + off[2];
  uint8_t* d3 = dst + off[3];
  for (size_t i = 0; i < q; ++i) {
    d0[i] = src[4 * i];
    d1[i] = src[4 * i + 1];
    d2[i] = src[4 * i + 2];
    d3[i] = src[4 * i + 3];
  }
  for (size_t g = 0; g < r; ++g) dst[off[g] + q] = src[4 * q + g];
}

void join(const uint8_t* src, size_t n, uint8_t* dst) {
  const size_t q = n / 4, r = n % 4;
  size_t off[4];
  off[0] = 0;
  for (int g = 1; g < 4; ++g) off[g] = off[g - 1] + q + (size_t(g - 1) < r ? 1 : 0);
  const uint8_t* s0 = src + off[0];
  const uint8_t* s1 = src + off[1];
  const uint8_t* s2 = src + off[2];
  const uint8_t* s3 = src + off[3];
  size_t i = 0;
  // 16 elements of each plane -> 64 interleaved bytes with byte then word unpacks (SSE2, baseline
  // x86-64): the scalar loop's four strided byte stores ran at ~5.8 GB/s
  for (; i + 16 <= q; i += 16) {
    const __m128i p0 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s0 + i));
    const __m128i p1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s1 + i));
    const __m128i p2 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s2 + i));
    const __m128i p3 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s3 + i));
    const __m128i a_lo = _mm_unpacklo_epi8(p0, p1), a_hi = _mm_unpackhi_epi8(p0, p1);
    const __m128i b_lo = _mm_unpacklo_epi8(p2, p3), b_hi = _mm_unpackhi_epi8(p2, p3);
    __m128i* d = reinterpret_cast<__m128i*>(dst + 4 * i);
    _mm_storeu_si128(d, _mm_unpacklo_epi16(a_lo, b_lo));
    _mm_storeu_si128(d + 1, _mm_unpackhi_epi16(a_lo, b_lo));
    _mm_storeu_si128(d + 2, _mm_unpacklo_epi16(a_hi, b_hi));
    _mm_storeu_si128(d + 3, _mm_unpackhi_epi16(a_hi, b_hi));
  }
  for (; i < q; ++i) {
    dst[4 * i] = s0[i];
    dst[4 * i + 1] = s1[i];
    dst[4 * i + 2] = s2[i];
    dst[4 * i + 3] = s3[i];
  }
  for (size_t g = 0; g < r; ++g) dst[4 * q + g] = src[off[g] + q];
}

}  // namespace zest::bg4

namespace zest::xet {

Scheme compress_chunk(const uint8_t* data, size_t n, CompressionPolicy policy, Bytes& out) {
  out.clear();
  if (policy == CompressionPolicy::None || n == 0) {
    out.assign(data, data + n);
    return Scheme::None;
  }
  Bytes best;
  Scheme best_s = Scheme::None;
  if (policy == CompressionPolicy::LZ4 || policy == CompressionPolicy::Auto) {
    best = lz4::compress_frame(data, n);
    best_s = Scheme::LZ4;
  }
  if (policy == CompressionPolicy::BG4 || policy == CompressionPolicy::Auto) {
    Bytes grouped(n);
    bg4::split(data, n, grouped.data());
    Bytes c = lz4::compress_frame(grouped.data(), n);
    if (best_s == Scheme::None || c.size() < best.size()) {
      best = std::move(c);
      best_s = Scheme::BG4LZ4;
    }
  }
  if (best.size() >= n) {
    out.assign(data, data + n);
    return Scheme::None;
  }
  out = std::move(best);
  return best_s;
}

void decompress_chunk(Scheme s, const uint8_t* payload, size_t clen, uint8_t* out, size_t ulen) {
  switch (s) {
    case Scheme::None:
      if (clen != ulen) throw Error("CorruptChunk", "uncompressed chunk length mismatch");
      std::memcpy(out, payload, ulen);
      return;
    case Scheme::LZ4:
      lz4::decompress_frame_into(payload, clen, out, ulen);
      return;
    case Scheme::BG4LZ4: {
      // the planes go through a per-thread buffer (a fresh zero-filled vector per chunk cost a
      // malloc + 64 KiB memset next to a ~30 us decode)
      thread_local Bytes tmp;
      if (tmp.size() < ulen) tmp.resize(ulen);
      lz4::decompress_frame_into(payload, clen, tmp.data(), ulen);
      bg4::join(tmp.data(), ulen, out);
      return;
    }
  }
  throw Error("UnsupportedScheme", std::to_string(int(s)));
}

}  // namespace zest::xet
