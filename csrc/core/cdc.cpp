#include "cdc.h"

#include <algorithm>

#include "gear_table.h"

namespace zest::xet {

// Pinned semantics (tests/test_xet_golden.py, crafted files): the gear hash is a plain rolling hash
// over the whole stream (it depends only on the last 64 bytes, so resets are irrelevant), and a
// chunk ends after byte i when chunk_len >= min_size and (h & mask) == 0, or chunk_len == max_size.
// We skip hashing the first (min_size - 64) bytes of each chunk: the 64 bytes hashed before the
// first eligible position rebuild the exact full-window state.

uint64_t CdcParams::mask() const {
  uint64_t m = uint64_t(target - 1);
  return m << __builtin_clzll(m);
}

Chunker::Chunker(CdcParams p) : p_(p), mask_(p.mask()) {}

void Chunker::feed(const uint8_t* data, size_t n, std::vector<uint64_t>& ends) {
  constexpr size_t kWindow = 64;
  const size_t warm_start = p_.min_size - kWindow;  // first chunk offset that must be hashed
  size_t pos = 0;
  while (pos < n) {
    if (chunk_len_ < warm_start) {
      size_t skip = std::min<size_t>(warm_start - chunk_len_, n - pos);
      pos += skip;
      chunk_len_ += skip;
      h_ = 0;
      if (pos >= n) break;
    }
    // Warm-up: hash without checking until chunk_len reaches min_size - 1.
    uint64_t h = h_;
    while (pos < n && chunk_len_ + 1 < p_.min_size) {
      h = (h << 1) + kGearTable[data[pos++]];
      ++chunk_len_;
    }
    if (pos >= n) {
      h_ = h;
      break;
    }
    const size_t read_end = std::min<size_t>(n, pos + (p_.max_size - chunk_len_));
    bool cut = false;
    size_t i = pos;
    for (; i < read_end; ++i) {
      h = (h << 1) + kGearTable[data[i]];
      if ((h & mask_) == 0) {
        ++i;
        cut = true;
        break;
      }
    }
    chunk_len_ += i - pos;
    pos = i;
    if (chunk_len_ >= p_.max_size) cut = true;
    h_ = h;
    if (cut) {
      total_ += chunk_len_;
      ends.push_back(total_);
      chunk_len_ = 0;
      h_ = 0;
    }
  }
}

void Chunker::finish(std::vector<uint64_t>& ends) {
  if (chunk_len_ > 0) {
    total_ += chunk_len_;
    ends.push_back(total_);
    chunk_len_ = 0;
    h_ = 0;
  }
}

std::vector<uint64_t> chunk_ends(const uint8_t* data, size_t n, CdcParams p) {
  Chunker c(p);
  std::vector<uint64_t> ends;
  ends.reserve(n / p.target + 2);
  c.feed(data, n, ends);
  c.finish(ends);
  return ends;
}

uint64_t gear_window_hash(const uint8_t* data, size_t i) {
  uint64_t h = 0;
  const size_t start = i >= 63 ? i - 63 : 0;
  for (size_t k = start; k <= i; ++k) h = (h << 1) + kGearTable[data[k]];
  return h;
}

}  // namespace zest::xet

namespace zest::xet {

std::vector<uint64_t> select_boundaries(const uint64_t* cand, size_t n_cand, uint64_t n, size_t min_size,
                                        size_t max_size) {
  std::vector<uint64_t> ends;
  ends.reserve(n / (min_size + max_size) * 2 + 4);
  uint64_t s = 0;
  size_t k = 0;
  while (s < n) {
    while (k < n_cand && cand[k] < s + min_size) ++k;
    uint64_t e;
    if (k < n_cand && cand[k] - s <= max_size) {
      e = cand[k];
    } else {
      e = s + max_size;
    }
    if (e >= n) e = n;
    ends.push_back(e);
    s = e;
  }
  return ends;
}

}  // namespace zest::xet
