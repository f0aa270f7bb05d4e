#include "xorb.h"

#include <cstring>

namespace zest::xet {

namespace {
constexpr char kIdentXorb[7] = {'X', 'E', 'T', 'B', 'L', 'O', 'B'};
constexpr char kIdentHashes[7] = {'X', 'B', 'L', 'B', 'H', 'S', 'H'};
constexpr char kIdentBounds[7] = {'X', 'B', 'L', 'B', 'B', 'N', 'D'};
constexpr uint8_t kXorbVersion = 1;
constexpr uint8_t kHashesVersion = 0;
constexpr uint8_t kBoundsVersion = 1;
}  // namespace

void write_chunk_header(uint8_t* p, const ChunkHeader& h) {
  p[0] = h.version;
  store_le24(p + 1, h.clen);
  p[4] = uint8_t(h.scheme);
  store_le24(p + 5, h.ulen);
}

ChunkHeader read_chunk_header(const uint8_t* p) {
  ChunkHeader h;
  h.version = p[0];
  h.clen = load_le24(p + 1);
  h.scheme = Scheme(p[4]);
  h.ulen = load_le24(p + 5);
  if (h.version != kChunkHeaderVersion) throw Error("CorruptChunk", "unknown chunk header version");
  if (p[4] > 2) throw Error("UnsupportedScheme", std::to_string(int(p[4])));
  return h;
}

std::optional<XorbFooter> parse_footer(const uint8_t* data, size_t n, size_t* footer_start) {
  if (n < 4 + 8) return std::nullopt;
  const uint32_t info_len = load_le32(data + n - 4);
  if (size_t(info_len) + 4 > n || info_len < 40 + 8 + 4) return std::nullopt;
  const size_t st = n - 4 - info_len;
  const uint8_t* f = data + st;
  if (std::memcmp(f, kIdentXorb, 7) != 0) return std::nullopt;
  XorbFooter out;
  size_t i = 8;
  std::memcpy(out.xorb_hash.data(), f + i, 32);
  i += 32;
  auto need = [&](size_t k) {
    if (i + k > info_len) throw Error("CorruptXorb", "truncated footer");
  };
  need(12);
  if (std::memcmp(f + i, kIdentHashes, 7) != 0) throw Error("CorruptXorb", "missing hash section");
  i += 8;
  const uint32_t nc = load_le32(f + i);
  i += 4;
  need(size_t(nc) * 32);
  out.chunk_hashes.resize(nc);
  for (uint32_t k = 0; k < nc; ++k, i += 32) std::memcpy(out.chunk_hashes[k].data(), f + i, 32);
  need(12);
  if (std::memcmp(f + i, kIdentBounds, 7) != 0) throw Error("CorruptXorb", "missing boundary section");
  i += 8;
  const uint32_t nc2 = load_le32(f + i);
  i += 4;
  if (nc2 != nc) throw Error("CorruptXorb", "chunk count mismatch");
  need(size_t(nc) * 8);
  out.chunk_boundaries.resize(nc);
  out.unpacked_offsets.resize(nc);
  for (uint32_t k = 0; k < nc; ++k, i += 4) out.chunk_boundaries[k] = load_le32(f + i);
  for (uint32_t k = 0; k < nc; ++k, i += 4) out.unpacked_offsets[k] = load_le32(f + i);
  if (footer_start) *footer_start = st;
  return out;
}

Bytes serialize_footer(const XorbFooter& f) {
  const uint32_t nc = uint32_t(f.chunk_hashes.size());
  Bytes out;
  append(out, kIdentXorb, 7);
  out.push_back(kXorbVersion);
  append(out, f.xorb_hash.data(), 32);
  const size_t hash_sec = out.size();
  append(out, kIdentHashes, 7);
  out.push_back(kHashesVersion);
  uint8_t w[4];
  store_le32(w, nc);
  append(out, w, 4);
  for (const auto& h : f.chunk_hashes) append(out, h.data(), 32);
  const size_t bound_sec = out.size();
  append(out, kIdentBounds, 7);
  out.push_back(kBoundsVersion);
  append(out, w, 4);
  for (uint32_t v : f.chunk_boundaries) {
    store_le32(w, v);
    append(out, w, 4);
  }
  for (uint32_t v : f.unpacked_offsets) {
    store_le32(w, v);
    append(out, w, 4);
  }
  // Trailer: num_chunks, section offsets measured back from the end of the info block,
  // 16 reserved bytes, then info_length.
  const size_t info_len = out.size() + 4 + 4 + 4 + 16;
  store_le32(w, nc);
  append(out, w, 4);
  store_le32(w, uint32_t(info_len - hash_sec));
  append(out, w, 4);
  store_le32(w, uint32_t(info_len - bound_sec));
  append(out, w, 4);
  uint8_t zeros[16] = {0};
  append(out, zeros, 16);
  store_le32(w, uint32_t(info_len));
  append(out, w, 4);
  return out;
}

std::vector<ChunkEntry> index_chunks(const uint8_t* data, size_t n) {
  size_t limit = n;
  size_t fst = 0;
  if (parse_footer(data, n, &fst)) limit = fst;
  std::vector<ChunkEntry> out;
  size_t p = 0;
  uint64_t unpacked = 0;
  while (p < limit) {
    if (limit - p < kChunkHeaderLen) throw Error("CorruptXorb", "truncated chunk header");
    ChunkHeader h = read_chunk_header(data + p);
    if (h.clen > limit - p - kChunkHeaderLen) throw Error("CorruptXorb", "chunk payload out of range");
    out.push_back({p, h.clen, h.scheme, h.ulen, unpacked});
    unpacked += h.ulen;
    p += kChunkHeaderLen + h.clen;
  }
  return out;
}

void extract_chunk_range(const uint8_t* data, size_t n, uint32_t start, uint32_t end, Bytes& out,
                         std::vector<HashSize>* hashes) {
  std::vector<ChunkEntry> idx = index_chunks(data, n);
  if (start > end || end > idx.size()) throw Error("RangeOutOfBounds");
  uint64_t total = 0;
  for (uint32_t i = start; i < end; ++i) total += idx[i].ulen;
  size_t base = out.size();
  out.resize(base + total);
  uint8_t* dst = out.data() + base;
  for (uint32_t i = start; i < end; ++i) {
    const ChunkEntry& e = idx[i];
    decompress_chunk(e.scheme, data + e.header_off + kChunkHeaderLen, e.clen, dst, e.ulen);
    if (hashes) hashes->push_back({chunk_hash(dst, e.ulen), e.ulen});
    dst += e.ulen;
  }
}

void verify_xorb(const uint8_t* data, size_t n, const Hash* expected) {
  auto footer = parse_footer(data, n);
  std::vector<ChunkEntry> idx = index_chunks(data, n);
  std::vector<HashSize> leaves;
  leaves.reserve(idx.size());
  Bytes tmp;
  for (size_t i = 0; i < idx.size(); ++i) {
    const ChunkEntry& e = idx[i];
    tmp.resize(e.ulen);
    decompress_chunk(e.scheme, data + e.header_off + kChunkHeaderLen, e.clen, tmp.data(), e.ulen);
    Hash h = chunk_hash(tmp.data(), e.ulen);
    if (footer && (i >= footer->chunk_hashes.size() || footer->chunk_hashes[i] != h))
      throw Error("HashMismatch", "chunk " + std::to_string(i));
    leaves.push_back({h, e.ulen});
  }
  Hash root = merkle_root(leaves);
  const Hash* want = expected ? expected : (footer ? &footer->xorb_hash : nullptr);
  if (want && *want != root) throw Error("HashMismatch", "xorb root");
}

bool XorbBuilder::fits(size_t ulen) const {
  return hashes_.size() + 1 <= kMaxXorbChunks &&
         body_.size() + kChunkHeaderLen + lz4::block_bound(ulen) + 64 <= kMaxXorbBytes;
}

uint32_t XorbBuilder::add_chunk(const uint8_t* data, size_t n) {
  Hash h = chunk_hash(data, n);
  Scheme s = compress_chunk(data, n, policy_, scratch_);
  return add_compressed(h, s, scratch_.data(), scratch_.size(), uint32_t(n));
}

uint32_t XorbBuilder::add_compressed(const Hash& h, Scheme s, const uint8_t* payload, size_t clen,
                                     uint32_t ulen) {
  uint8_t hdr[kChunkHeaderLen];
  write_chunk_header(hdr, {kChunkHeaderVersion, uint32_t(clen), s, ulen});
  append(body_, hdr, kChunkHeaderLen);
  append(body_, payload, clen);
  hashes_.push_back(h);
  ulens_.push_back(ulen);
  bounds_.push_back(uint32_t(body_.size()));
  unpacked_ += ulen;
  unpacked_ends_.push_back(uint32_t(unpacked_));
  return uint32_t(hashes_.size() - 1);
}

Hash XorbBuilder::hash() const {
  std::vector<HashSize> leaves(hashes_.size());
  for (size_t i = 0; i < hashes_.size(); ++i) leaves[i] = {hashes_[i], ulens_[i]};
  return merkle_root(leaves);
}

Bytes XorbBuilder::serialize(bool with_footer) const {
  Bytes out = body_;
  if (with_footer) {
    XorbFooter f{hash(), hashes_, bounds_, unpacked_ends_};
    Bytes foot = serialize_footer(f);
    out.insert(out.end(), foot.begin(), foot.end());
  }
  return out;
}

void XorbBuilder::clear() {
  body_.clear();
  hashes_.clear();
  ulens_.clear();
  bounds_.clear();
  unpacked_ends_.clear();
  unpacked_ = 0;
}

}  // namespace zest::xet
