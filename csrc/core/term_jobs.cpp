#include "term_jobs.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "lz4.h"
#include "trace.h"
#include "xet_hash.h"
#include "xorb.h"

namespace zest {

const cas::Reconstruction& ReconCache::get(const std::string& hex) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = recs_.find(hex);
    if (it != recs_.end()) return it->second;
  }
  // Outside the lock: several files' reconstructions may be requested concurrently.  std::map
  // nodes are stable, so a reference handed out earlier survives later inserts.
  cas::Reconstruction r = bridge_.get_reconstruction(hex);
  if (r.offset_into_first_range != 0) throw Error("Unsupported", "partial-file reconstruction of " + hex);
  std::lock_guard<std::mutex> g(mu_);
  return recs_.emplace(hex, std::move(r)).first->second;
}

std::vector<TermShape> ReconCache::shapes(const std::string& hex) {
  const cas::Reconstruction& r = get(hex);
  std::vector<TermShape> out;
  out.reserve(r.terms.size());
  for (const auto& t : r.terms) out.push_back({t.unpacked_length, uint32_t(t.range.end - t.range.start)});
  return out;
}

std::vector<TermKey> ReconCache::keys(const std::string& hex) {
  const cas::Reconstruction& r = get(hex);
  std::vector<TermKey> out;
  out.reserve(r.terms.size());
  for (const auto& t : r.terms) out.push_back({t.hash_hex, uint32_t(t.range.start), uint32_t(t.range.end)});
  return out;
}

void ReconCache::clear() {
  std::lock_guard<std::mutex> g(mu_);
  recs_.clear();
}

std::vector<uint8_t> cached_terms(const storage::XorbCache& cache, const std::vector<std::string>& hexes,
                                  const std::vector<uint32_t>& starts, const std::vector<uint32_t>& ends, int threads) {
  const size_t n = hexes.size();
  if (starts.size() != n || ends.size() != n) throw Error("InvalidArgument", "cached_terms: lists of different lengths");
  std::vector<uint8_t> out(n, 0);
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < n;) {
      try {
        out[i] = cache.covers(hexes[i], starts[i], ends[i]) ? 1 : 0;
      } catch (const std::exception&) {
        out[i] = 0;
      }
    }
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < std::max(1, std::min<int>(threads, int(n))); ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  return out;
}

void SettleBook::add(const std::string& file_hex, const std::string& xorb_hex, Source src, uint32_t run_offset,
                     const std::string& pending) {
  // Only runs with something to settle: a quarantined peer run, or a cache hit (evicted on failure).
  if (pending.empty() && src != Source::Cache) return;
  std::lock_guard<std::mutex> g(mu_);
  runs_[file_hex].push_back({xorb_hex, src, run_offset, pending});
}

size_t SettleBook::settle(XetBridge& bridge, const std::string& file_hex, bool ok) {
  std::vector<Run> runs;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = runs_.find(file_hex);
    if (it == runs_.end()) return 0;
    runs = std::move(it->second);
    runs_.erase(it);
  }
  for (const Run& r : runs) bridge.settle(r.xorb_hex, r.src, r.run_offset, r.pending, ok);
  return runs.size();
}

size_t SettleBook::discard(XetBridge& bridge, const std::vector<std::pair<std::string, std::string>>& runs) {
  std::vector<Run> gone;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& [file, pending] : runs) {
      auto it = runs_.find(file);
      if (it == runs_.end()) continue;
      auto& v = it->second;
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i].pending == pending) {
          gone.push_back(std::move(v[i]));
          v.erase(v.begin() + long(i));
          break;
        }
    }
  }
  for (const Run& r : gone) bridge.settle(r.xorb_hex, r.src, r.run_offset, r.pending, false);
  return gone.size();
}

size_t SettleBook::settle_all(XetBridge& bridge, bool ok) {
  std::vector<std::string> files;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : runs_) files.push_back(kv.first);
  }
  size_t n = 0;
  for (auto& f : files) n += settle(bridge, f, ok);
  return n;
}

std::vector<TermJobResult> fetch_terms_host(XetBridge& bridge, ReconCache& recs, SettleBook& book,
                                            const std::vector<TermJob>& jobs, uint8_t* hashes, int threads,
                                            bool repair) {
  // Flatten the jobs into (job, term, output offset, chunk index) work items.
  struct Item {
    size_t job;
    uint32_t term;
    uint64_t out_off;  // from the job's dst
    uint64_t chunk;    // global chunk index
    uint32_t lens_at;  // position of the term's first chunk in the job's chunk_lens
  };
  std::vector<const cas::Reconstruction*> rec_of(jobs.size());
  std::vector<Item> items;
  std::vector<TermJobResult> out(jobs.size());
  for (size_t j = 0; j < jobs.size(); ++j) {
    const TermJob& jb = jobs[j];
    rec_of[j] = &recs.get(jb.xet_hash);
    const auto& terms = rec_of[j]->terms;
    if (jb.t0 > jb.t1 || jb.t1 > terms.size()) throw Error("RangeOutOfBounds", "term range of " + jb.xet_hash);
    uint64_t off = 0, c = jb.chunk0;
    uint32_t at = 0;
    for (uint32_t t = jb.t0; t < jb.t1; ++t) {
      const uint32_t n = uint32_t(terms[t].range.end - terms[t].range.start);
      items.push_back({j, t, off, c, at});
      off += terms[t].unpacked_length;
      c += n;
      at += n;
    }
    out[j].chunk_lens.assign(at, 0);
  }
  std::atomic<size_t> next{0};
  std::atomic<bool> failed{false};
  std::mutex mu;
  std::string first_err;
  std::vector<std::pair<std::string, std::string>> quarantined;  // (file, pending) added by this call
  auto do_term = [&](const Item& it, const FetchOptions& opt, Source* src_out, std::string* peer_out) {
    const cas::Reconstruction& rec = *rec_of[it.job];
    const cas::Term& t = rec.terms[it.term];
    XorbFetchResult f = bridge.fetch_term(t, rec, opt);
    *src_out = f.source;
    *peer_out = f.peer;
    // The run's cache bookkeeping is recorded before decoding, so a copy that fails to decode is
    // still rejected (its quarantine dropped) by the caller.
    bool recorded = false;
    auto record = [&](bool ok_now) {
      if (recorded) return;
      recorded = true;
      if (ok_now) {
        book.add(jobs[it.job].xet_hash, t.hash_hex, f.source, f.run_offset, f.pending);
        if (!f.pending.empty()) {
          std::lock_guard<std::mutex> g(mu);
          quarantined.emplace_back(jobs[it.job].xet_hash, f.pending);
        }
      } else {
        bridge.settle(t.hash_hex, f.source, f.run_offset, f.pending, false);
      }
    };
    try {
      const auto idx = xet::index_chunks(f.bytes(), f.size());
      if (f.local_start > f.local_end || f.local_end > idx.size() ||
          f.local_end - f.local_start != t.range.end - t.range.start)
        throw Error("RangeOutOfBounds", t.hash_hex);
      uint8_t* dst = reinterpret_cast<uint8_t*>(jobs[it.job].dst) + it.out_off;
      uint64_t total = 0;
      TermJobResult& res = out[it.job];
      for (uint32_t c = f.local_start; c < f.local_end; ++c) {
        const xet::ChunkEntry& e = idx[c];
        if (total + e.ulen > t.unpacked_length) throw Error("SizeMismatch", "term larger than planned");
        const uint8_t* payload = f.bytes() + e.header_off + xet::kChunkHeaderLen;
        if (e.scheme != xet::Scheme::None) {
          xet::decompress_chunk(e.scheme, payload, e.clen, dst + total, e.ulen);
        } else {
          if (e.clen != e.ulen) throw Error("CorruptChunk", "stored chunk length mismatch");
          std::memcpy(dst + total, payload, e.ulen);
        }
        const xet::Hash h = xet::chunk_hash(dst + total, e.ulen);
        std::memcpy(hashes + 32 * (it.chunk + (c - f.local_start)), h.data(), 32);
        res.chunk_lens[it.lens_at + (c - f.local_start)] = e.ulen;
        total += e.ulen;
      }
      if (total != t.unpacked_length) throw Error("SizeMismatch", "term " + std::to_string(it.term));
      record(true);
      std::lock_guard<std::mutex> g(mu);
      res.fetched += f.size();
      (f.source == Source::Peer ? res.from_peer : f.source == Source::Cache ? res.from_cache : res.from_cdn) += total;
    } catch (...) {
      record(false);
      throw;
    }
  };
  auto worker = [&]() {
    while (!failed.load()) {
      const size_t i = next.fetch_add(1);
      if (i >= items.size()) return;
      Source src = Source::Cdn;
      std::string peer;
      try {
        do_term(items[i], FetchOptions{true, true, repair}, &src, &peer);
      } catch (const std::exception& e) {
        ZTRACE("download", "term " << items[i].term << " failed (" << e.what() << "), CDN retry");
        if (src == Source::Peer && !peer.empty() && bridge.swarm()) bridge.swarm()->report_bad_peer(peer);
        try {
          do_term(items[i], FetchOptions{false, false, src != Source::Cdn || repair}, &src, &peer);
        } catch (const std::exception& e2) {
          std::lock_guard<std::mutex> g(mu);
          if (first_err.empty()) first_err = e2.what();
          failed = true;
        }
      }
    }
  };
  const int nt = std::max(1, std::min<int>(threads > 0 ? threads : 16, int(items.size())));
  std::vector<std::thread> ts;
  for (int k = 1; k < nt; ++k) ts.emplace_back(worker);
  worker();
  for (auto& t : ts) t.join();
  if (failed) {
    // The range is refetched by another rank: drop only the peer runs this call quarantined (they
    // will never be Merkle-checked); cache hits and earlier calls' runs wait for the file's verdict.
    book.discard(bridge, quarantined);
    throw Error("DownloadFailed", first_err);
  }
  return out;
}

std::vector<std::pair<uint64_t, uint64_t>> copy_ranges(const std::vector<uint64_t>& at,
                                                       const std::vector<uint64_t>& len, uint64_t max_gap) {
  std::vector<std::pair<uint64_t, uint64_t>> r;
  for (size_t i = 0; i < at.size() && i < len.size(); ++i)
    if (len[i]) r.emplace_back(at[i], at[i] + len[i]);
  std::sort(r.begin(), r.end());
  std::vector<std::pair<uint64_t, uint64_t>> out;
  for (const auto& x : r) {
    if (!out.empty() && x.first <= out.back().second + max_gap) out.back().second = std::max(out.back().second, x.second);
    else out.push_back(x);
  }
  return out;
}

}  // namespace zest
