#include "downloader.h"

#include <fcntl.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <optional>
#include <thread>

#include "lz4.h"
#include "storage.h"
#include "trace.h"
#include "xorb.h"

namespace zest {

namespace {

constexpr char kResumeMagic[4] = {'Z', 'R', 'S', '1'};

struct Sidecar {
  int fd = -1;
  std::mutex mu;
  ~Sidecar() {
    if (fd >= 0) ::close(fd);
  }
  void append(uint32_t term, const std::vector<xet::HashSize>& hs) {
    Bytes rec(8 + hs.size() * 40);
    store_le32(rec.data(), term);
    store_le32(rec.data() + 4, uint32_t(hs.size()));
    for (size_t i = 0; i < hs.size(); ++i) {
      std::memcpy(rec.data() + 8 + 40 * i, hs[i].hash.data(), 32);
      store_le64(rec.data() + 8 + 40 * i + 32, hs[i].size);
    }
    std::lock_guard<std::mutex> g(mu);
    if (::write(fd, rec.data(), rec.size()) != ssize_t(rec.size())) throw Error("IoError", "resume sidecar");
  }
};

void pwrite_all(int fd, const uint8_t* p, size_t n, uint64_t off) {
  while (n) {
    ssize_t w = ::pwrite(fd, p, n, off_t(off));
    if (w < 0) {
      if (errno == EINTR) continue;
      throw Error("IoError", std::string("pwrite: ") + std::strerror(errno));
    }
    p += w;
    n -= size_t(w);
    off += uint64_t(w);
  }
}

// Run fn(part) for part in [0, parts) on parts - 1 extra threads + the caller; rethrows the first
// exception.  Used inside one term: when the swarm's last terms land together (striped peers finish
// at the same moment), their decode/hash/write is the whole tail of a pull, and one thread per term
// leaves the other cores idle.
template <class F>
void run_parts(int parts, F&& fn) {
  if (parts <= 1) {
    fn(0);
    return;
  }
  std::vector<std::exception_ptr> errs(static_cast<size_t>(parts));
  std::vector<std::thread> ts;
  for (int k = 1; k < parts; ++k)
    ts.emplace_back([&, k] {
      try {
        fn(k);
      } catch (...) {
        errs[size_t(k)] = std::current_exception();
      }
    });
  try {
    fn(0);
  } catch (...) {
    errs[0] = std::current_exception();
  }
  for (auto& t : ts) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// Threads per large term (ZEST_TERM_THREADS, default 4; terms under 128 chunks use one).
int term_threads(size_t chunks) {
  static const int n = [] {
    const char* e = std::getenv("ZEST_TERM_THREADS");
    const int v = e ? std::atoi(e) : 4;
    return std::max(1, std::min(v, 16));
  }();
  return chunks >= 128 ? std::min<int>(n, int(chunks / 64)) : 1;
}

// pwritev of the whole list (IOV_MAX-sized batches, partial writes resumed).
void pwritev_all(int fd, std::vector<iovec>& iov, uint64_t off) {
  size_t k = 0;
  while (k < iov.size()) {
    const int cnt = int(std::min<size_t>(iov.size() - k, 1024));
    ssize_t w = ::pwritev(fd, iov.data() + k, cnt, off_t(off));
    if (w < 0) {
      if (errno == EINTR) continue;
      throw Error("IoError", std::string("pwritev: ") + std::strerror(errno));
    }
    off += uint64_t(w);
    size_t left = size_t(w);
    while (k < iov.size() && left >= iov[k].iov_len) left -= iov[k++].iov_len;
    if (k < iov.size() && left) {
      iov[k].iov_base = static_cast<uint8_t*>(iov[k].iov_base) + left;
      iov[k].iov_len -= left;
    }
  }
}

}  // namespace

ParallelDownloader::RunBuffer* ParallelDownloader::acquire_slot() {
  std::unique_lock<std::mutex> g(gate_mu_);
  gate_cv_.wait(g, [&] { return free_ > 0; });
  --free_;
  RunBuffer* b = bufs_.back().release();
  bufs_.pop_back();
  return b;
}

void ParallelDownloader::release_slot(RunBuffer* b) {
  {
    std::lock_guard<std::mutex> g(gate_mu_);
    bufs_.emplace_back(b);
    ++free_;
  }
  gate_cv_.notify_one();
}

FileResult ParallelDownloader::reconstruct_to_file(const std::string& hex, const std::string& out_path, bool verify,
                                                   const std::function<void(uint64_t, Source)>& on_term) {
  return reconstruct(hex, out_path, nullptr, 0, verify, on_term);
}

FileResult ParallelDownloader::reconstruct_to_memory(const std::string& hex, uint8_t* dst, uint64_t cap, bool verify,
                                                     const std::function<void(uint64_t, Source)>& on_term) {
  if (!dst && cap) throw Error("InvalidArgument", "null destination");
  return reconstruct(hex, std::string(), dst, cap, verify, on_term);
}

FileResult ParallelDownloader::reconstruct(const std::string& hex, const std::string& out_path, uint8_t* mem,
                                           uint64_t mem_cap, bool verify,
                                           const std::function<void(uint64_t, Source)>& on_term) {
  const bool to_mem = out_path.empty();
  const auto t0 = std::chrono::steady_clock::now();
  std::optional<trace::Span> rec_span(std::in_place, "download", "get_reconstruction");
  cas::Reconstruction rec = bridge_.get_reconstruction(hex);
  rec_span.reset();
  const size_t n = rec.terms.size();
  std::vector<uint64_t> offs(n + 1, 0);
  for (size_t i = 0; i < n; ++i) offs[i + 1] = offs[i] + rec.terms[i].unpacked_length;
  const uint64_t skip = rec.offset_into_first_range;
  const uint64_t total = offs[n] - skip;
  if (to_mem && total > mem_cap) throw Error("SizeMismatch", "file " + hex + " is larger than its buffer");
  const size_t slash = out_path.rfind('/');
  if (!to_mem && slash != std::string::npos) storage::ensure_dir(out_path.substr(0, slash));
  const std::string tmp = to_mem ? std::string() : out_path + ".incomplete";
  const std::string side = to_mem ? std::string() : out_path + ".zest-resume";

  std::vector<std::vector<xet::HashSize>> hashes(n);
  std::vector<uint8_t> done(n, 0);
  // Where each term's bytes came from, and the cache run behind them (for settle()).
  std::vector<Source> src(n, Source::Cdn);
  std::vector<std::string> peer(n);
  std::vector<uint32_t> run_off(n, 0);
  std::vector<std::string> pending(n);  // quarantine file of a peer run, until settled
  size_t resumed = 0;
  // ---- resume from sidecar
  if (!to_mem && storage::exists(tmp) && storage::exists(side)) {
    if (auto b = storage::read_file(side); b && b->size() >= 4 + 64 + 4 && std::memcmp(b->data(), kResumeMagic, 4) == 0 &&
                                         std::string(reinterpret_cast<char*>(b->data()) + 4, 64) == hex &&
                                         load_le32(b->data() + 68) == n) {
      size_t p = 72;
      while (p + 8 <= b->size()) {
        const uint32_t t = load_le32(b->data() + p), k = load_le32(b->data() + p + 4);
        if (t >= n || p + 8 + size_t(k) * 40 > b->size()) break;
        std::vector<xet::HashSize> hs(k);
        for (uint32_t i = 0; i < k; ++i) {
          std::memcpy(hs[i].hash.data(), b->data() + p + 8 + 40 * i, 32);
          hs[i].size = load_le64(b->data() + p + 8 + 40 * i + 32);
        }
        hashes[t] = std::move(hs);
        if (!done[t]) ++resumed;
        src[t] = Source::Resumed;
        done[t] = 1;
        p += 8 + size_t(k) * 40;
      }
    }
  }
  if (!resumed && !to_mem) storage::remove_file(side);
  int fd = -1;
  Sidecar sc;
  if (!to_mem) {
    fd = ::open(tmp.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
    if (fd < 0) throw Error("IoError", tmp + ": " + std::strerror(errno));
    if (::ftruncate(fd, off_t(total)) != 0) {
      ::close(fd);
      throw Error("IoError", "ftruncate");
    }
  }
  const bool fresh = !to_mem && !storage::exists(side);
  if (!to_mem) sc.fd = ::open(side.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (sc.fd >= 0 && fresh) {
    Bytes h(72);
    std::memcpy(h.data(), kResumeMagic, 4);
    std::memcpy(h.data() + 4, hex.data(), 64);
    store_le32(h.data() + 68, uint32_t(n));
    if (::write(sc.fd, h.data(), h.size()) != 72) throw Error("IoError", "resume header");
  }

  std::atomic<size_t> next{0};
  std::atomic<bool> failed{false};
  std::string first_err;
  std::mutex err_mu;

  // A term's earlier copy failed (decode error or file hash): drop/evict the cached run behind
  // it and blame the peer that served it.
  auto reject = [&](size_t i) {
    if (src[i] == Source::Peer && !peer[i].empty() && bridge_.swarm()) bridge_.swarm()->report_bad_peer(peer[i]);
    bridge_.settle(rec.terms[i].hash_hex, src[i], run_off[i], pending[i], false);
    pending[i].clear();
  };
  auto do_term = [&](size_t i, const FetchOptions& opt, RunBuffer* buf) {
    const cas::Term& t = rec.terms[i];
    XorbFetchResult f = bridge_.fetch_term(t, rec, opt, [buf](size_t nbytes) { return buf->get(nbytes); });
    src[i] = f.source;  // recorded before decoding so a bad peer copy can be attributed
    peer[i] = f.peer;
    run_off[i] = f.run_offset;
    pending[i] = f.pending;
    // Uncompressed chunks are hashed and written straight from the fetched run (no decode
    // buffer); compressed ones are decoded into one buffer for the term.
    std::vector<xet::HashSize> hs;
    std::vector<iovec> iov;
    Bytes dec;
    uint64_t total = 0;
    int parts = 1;
    {
      trace::Span sp("download", "decode+hash");
      const auto idx = xet::index_chunks(f.bytes(), f.size());
      if (f.local_start > f.local_end || f.local_end > idx.size()) throw Error("RangeOutOfBounds");
      const size_t nc = f.local_end - f.local_start;
      // each compressed chunk's place in the decode buffer (prefix sum), so parts decode independently
      std::vector<uint64_t> dpos(nc + 1, 0);
      for (size_t k = 0; k < nc; ++k) {
        const xet::ChunkEntry& e = idx[f.local_start + k];
        dpos[k + 1] = dpos[k] + (e.scheme != xet::Scheme::None ? e.ulen : 0);
        total += e.ulen;
      }
      dec.resize(dpos[nc]);
      hs.resize(nc);
      iov.resize(nc);
      parts = term_threads(nc);
      sp.arg("\"threads\":" + std::to_string(parts));
      run_parts(parts, [&](int part) {
        for (size_t k = nc * size_t(part) / size_t(parts); k < nc * size_t(part + 1) / size_t(parts); ++k) {
          const xet::ChunkEntry& e = idx[f.local_start + k];
          const uint8_t* payload = f.bytes() + e.header_off + xet::kChunkHeaderLen;
          const uint8_t* p = payload;
          if (e.scheme != xet::Scheme::None) {
            uint8_t* dp = dec.data() + dpos[k];
            xet::decompress_chunk(e.scheme, payload, e.clen, dp, e.ulen);
            p = dp;
          } else if (e.clen != e.ulen) {
            throw Error("CorruptChunk", "stored chunk length mismatch");
          }
          hs[k] = {xet::chunk_hash(p, e.ulen), e.ulen};
          iov[k] = {const_cast<uint8_t*>(p), e.ulen};
        }
      });
    }
    if (total != t.unpacked_length) throw Error("SizeMismatch", "term " + std::to_string(i));
    uint64_t off = offs[i];
    if (off < skip) {  // only the first term can straddle offset_into_first_range
      uint64_t drop = std::min<uint64_t>(skip - off, total);
      size_t k = 0;
      while (k < iov.size() && drop >= iov[k].iov_len) drop -= iov[k++].iov_len;
      iov.erase(iov.begin(), iov.begin() + long(k));
      if (!iov.empty() && drop) {
        iov[0].iov_base = static_cast<uint8_t*>(iov[0].iov_base) + drop;
        iov[0].iov_len -= drop;
      }
      off = skip;
    }
    if (to_mem) {
      trace::Span sp("download", "copy");
      uint64_t o = off - skip;
      for (const iovec& v : iov) {
        if (o + v.iov_len > mem_cap) throw Error("SizeMismatch", "term past the end of the buffer");
        std::memcpy(mem + o, v.iov_base, v.iov_len);
        o += v.iov_len;
      }
    } else {
      trace::Span sp("download", "pwrite");
      uint64_t n = 0;
      for (const iovec& v : iov) n += v.iov_len;
      // the term's chunks in `parts` contiguous groups, written concurrently at their own offsets
      const int wp = std::min<int>(parts, int(iov.size()));
      std::vector<uint64_t> at(size_t(wp) + 1, off - skip);
      std::vector<std::vector<iovec>> groups(static_cast<size_t>(wp));
      for (int g = 0; g < wp; ++g) {
        const size_t a = iov.size() * size_t(g) / size_t(wp), b = iov.size() * size_t(g + 1) / size_t(wp);
        groups[size_t(g)].assign(iov.begin() + long(a), iov.begin() + long(b));
        uint64_t len = 0;
        for (size_t k = a; k < b; ++k) len += iov[k].iov_len;
        at[size_t(g) + 1] = at[size_t(g)] + len;
      }
      if (wp > 0) run_parts(wp, [&](int g) { pwritev_all(fd, groups[size_t(g)], at[size_t(g)]); });
      storage::start_writeback(fd, off - skip, n);
    }
    hashes[i] = std::move(hs);
    if (on_term) on_term(total, f.source);
  };

  auto worker = [&]() {
    while (!failed.load()) {
      const size_t i = next.fetch_add(1);
      if (i >= n) return;
      if (done[i]) continue;
      struct Slot {
        ParallelDownloader* d;
        RunBuffer* buf;
        ~Slot() { d->release_slot(buf); }
      } slot{this, acquire_slot()};
      try {
        do_term(i, FetchOptions{}, slot.buf);
        if (sc.fd >= 0) sc.append(uint32_t(i), hashes[i]);
      } catch (const std::exception& e) {
        // A peer/cache copy that does not decode: retry straight from the CDN once.
        ZTRACE("download", "term " << i << " via " << int(src[i]) << " failed (" << e.what() << "), CDN retry");
        try {
          if (src[i] != Source::Cdn) reject(i);
          do_term(i, FetchOptions{false, false, /*repair=*/src[i] != Source::Cdn}, slot.buf);
          if (sc.fd >= 0) sc.append(uint32_t(i), hashes[i]);
        } catch (const std::exception& e2) {
          std::lock_guard<std::mutex> g(err_mu);
          if (first_err.empty()) first_err = e2.what();
          failed = true;
        }
      }
    }
  };
  const int nthreads = std::max(1, std::min<int>(concurrency_, int(n)));
  std::vector<std::thread> ts;
  for (int k = 0; k < nthreads; ++k) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
  auto close_fd = [&] {
    if (fd >= 0) ::close(fd);
    fd = -1;
  };
  if (failed) {
    close_fd();
    for (size_t i = 0; i < n; ++i)
      if (!pending[i].empty()) bridge_.settle(rec.terms[i].hash_hex, src[i], run_off[i], pending[i], false);
    throw Error("DownloadFailed", first_err);
  }
  bool ok = true;
  if (verify) {
    auto file_hash_now = [&]() {
      std::vector<xet::HashSize> leaves;
      for (auto& h : hashes) leaves.insert(leaves.end(), h.begin(), h.end());
      return xet::to_hex(xet::file_hash(leaves));
    };
    {
      trace::Span vs("download", "file hash verify");
      ok = file_hash_now() == hex;
    }
    if (!ok) {
      // Repair: every term not fetched from the CDN in this run — peer runs, cache hits and terms
      // restored from the resume sidecar — is refetched from the CDN, replacing its cached copy.
      bridge_.stats().verify_failures++;
      RunBuffer repair_buf;
      try {
        for (size_t i = 0; i < n; ++i) {
          if (src[i] == Source::Cdn) continue;
          reject(i);
          do_term(i, FetchOptions{false, false, /*repair=*/true}, &repair_buf);
          bridge_.stats().refetches++;
        }
      } catch (...) {  // the CDN failed too: keep the sidecar (resumed terms are re-checked next run)
        close_fd();
        for (size_t i = 0; i < n; ++i)
          if (!pending[i].empty()) bridge_.settle(rec.terms[i].hash_hex, src[i], run_off[i], pending[i], false);
        throw;
      }
      trace::Span vs("download", "file hash verify");
      ok = file_hash_now() == hex;
    }
    if (!ok) {
      close_fd();
      if (!to_mem) storage::remove_file(side);
      throw Error("HashMismatch", "file " + hex);
    }
  }
  // The file checked out (or the caller skipped verification): publish the quarantined peer runs.
  for (size_t i = 0; i < n; ++i)
    if (!pending[i].empty()) bridge_.settle(rec.terms[i].hash_hex, src[i], run_off[i], pending[i], true);
  FileResult r;
  if (to_mem) {
    for (auto& h : hashes)
      for (auto& x : h) r.chunk_lens.push_back(uint32_t(x.size));
  } else {
    {
      trace::Span sp("download", "fdatasync");  // (the disk's share of a pull's wall time)
      ::fdatasync(fd);
    }
    close_fd();
    if (::rename(tmp.c_str(), out_path.c_str()) != 0) throw Error("IoError", "rename " + out_path);
    storage::remove_file(side);
  }
  r.bytes = total;
  r.terms = n;
  r.resumed_terms = resumed;
  r.verified = verify && ok;
  r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

}  // namespace zest
