#include "bridge.h"

#include <tuple>

#include <algorithm>

#include <cstring>
#include <iomanip>

#include "json.h"
#include "trace.h"
#include "xorb.h"

namespace zest {

void XetBridge::authenticate(const std::string& repo_id, const std::string& repo_type, const std::string& revision) {
  hub::XetToken t = hub::xet_read_token(cfg_, repo_id, revision, repo_type);
  set_cas(t.cas_url, t.access_token);
}

void XetBridge::set_cas(const std::string& cas_url, const std::string& token) {
  cas_ = std::make_unique<cas::CasClient>(cas_url, token);
}

cas::Reconstruction XetBridge::get_reconstruction(const std::string& file_hash_hex) const {
  if (!cas_) throw Error("NotAuthenticated");
  return cas_->get_reconstruction(file_hash_hex);
}

namespace {
// A cached / received run must contain the term's chunks.
bool covers(const uint8_t* data, size_t n, uint32_t chunk_offset, uint64_t start, uint64_t end) {
  if (start < chunk_offset) return false;
  try {
    auto idx = xet::index_chunks(data, n);
    return end - chunk_offset <= idx.size();
  } catch (const Error&) {
    return false;
  }
}
}  // namespace

XorbFetchResult XetBridge::fetch_term(const cas::Term& term, const cas::Reconstruction& recon,
                                      const FetchOptions& opt, const bt::PayloadSink& sink) {
  // Copy a run into sink memory when the caller provided room for it; else keep it in `data`.
  auto land = [&](XorbFetchResult& out, const uint8_t* p, size_t n, Bytes* owned) {
    if (uint8_t* d = sink ? sink(n) : nullptr) {
      std::memcpy(d, p, n);
      out.ext = d;
      out.ext_len = n;
    } else if (owned) {
      out.data = std::move(*owned);
    } else {
      out.data.assign(p, p + n);
    }
  };
  const std::string& hex = term.hash_hex;
  auto it = recon.fetch_info.find(hex);
  if (it == recon.fetch_info.end()) throw Error("NotAuthenticated", "no fetch_info for " + hex);
  const cas::FetchInfo* fi = recon.match(hex, term.range.start, term.range.end);
  if (!fi) throw Error("NoMatchingFetchInfo", hex);
  XorbFetchResult out;
  // 1. local xorb cache: any cached run covering the term's chunks
  if (opt.allow_cache && !opt.repair && cache_ && cache_->maybe_cached(hex)) {
    trace::Span sp("cache", "find");
    if (auto hit = cache_->find(hex, uint32_t(term.range.start), uint32_t(term.range.end))) {
      stats_.xorbs_from_cache++;
      stats_.bytes_from_cache += hit->size();
      if (swarm_) swarm_->stats().cached_xorbs++;
      land(out, hit->bytes(), hit->size(), hit->ext ? nullptr : &hit->data);  // hits view a file mapping
      out.local_start = uint32_t(term.range.start - hit->chunk_offset);
      out.local_end = uint32_t(term.range.end - hit->chunk_offset);
      out.source = Source::Cache;
      out.run_offset = hit->run_offset;
      return out;
    }
  }
  // 2. P2P swarm with the FetchInfo's chunk range
  if (opt.allow_p2p && !opt.repair && swarm_ && swarm_->p2p_enabled()) {
    if (auto r = swarm_->try_peers(term.hash, uint32_t(fi->range.start), uint32_t(fi->range.end), sink)) {
      if (covers(r->bytes(), r->size(), r->chunk_offset, term.range.start, term.range.end)) {
        stats_.xorbs_from_peer++;
        stats_.bytes_from_peer += r->size();
        // Nothing has checked these bytes yet: quarantine the run until the caller verified the
        // file (settle), so a corrupt peer copy is never seeded on or read back as a cache hit.
        if (cache_ && cfg_.cache_writes) {
          try {
            if (writer_ && opt.on_copied && r->ext) {  // copied off this thread (sink memory stays put)
              out.pending = writer_->put_pending_ref(hex, r->chunk_offset, r->ext, r->ext_len, opt.on_copied);
              out.copy_deferred = !out.pending.empty();
            } else {
              trace::Span sp("cache", "put_pending");
              out.pending = writer_ ? writer_->put_pending(hex, r->chunk_offset, r->bytes(), r->size())
                                    : cache_->put_pending(hex, r->chunk_offset, r->bytes(), r->size());
            }
            if (writer_ && out.pending.empty()) defer(hex, *fi, false);  // the writer's queue was full
            out.run_offset = r->chunk_offset;
          } catch (const Error&) {
          }
        }
        out.local_start = uint32_t(term.range.start - r->chunk_offset);
        out.local_end = uint32_t(term.range.end - r->chunk_offset);
        if (r->ext) {
          out.ext = r->ext;
          out.ext_len = r->ext_len;
        } else {
          out.data = std::move(r->data);
        }
        out.source = Source::Peer;
        out.peer = r->peer;
        return out;
      }
      ZTRACE("bridge", "peer " << r->peer << " run for " << hex << " does not cover [" << term.range.start << ","
                                << term.range.end << ") (offset " << r->chunk_offset << ")");
      swarm_->report_bad_peer(r->peer);  // served a run that does not even parse
    }
  }
  // 3. CDN: straight into the sink's memory when it has room (no intermediate buffer)
  if (!cas_) throw Error("NotAuthenticated");
  trace::Span span("cdn", "fetch " + hex.substr(0, 12));
  const size_t want = size_t(fi->url_range.end - fi->url_range.start + 1);
  Bytes body;
  const uint8_t* run = nullptr;
  size_t run_len = 0;
  if (uint8_t* d = sink ? sink(want) : nullptr) {
    if (size_t n = cas_->fetch_into(*fi, d, want)) {
      run = d;
      run_len = n;
      out.ext = d;
      out.ext_len = n;
    }
  }
  if (!run) {
    body = cas_->fetch(*fi);
    run = body.data();
    run_len = body.size();
  }
  span.arg("\"bytes\":" + std::to_string(run_len));
  stats_.xorbs_from_cdn++;
  stats_.bytes_from_cdn += run_len;
  if (swarm_) {
    swarm_->stats().cdn_xorbs++;
    swarm_->stats().total_xorbs++;
    swarm_->stats().total_bytes += run_len;
  }
  if (cache_ && cfg_.cache_writes) {
    try {
      if (writer_ && opt.on_copied && out.ext) {
        out.copy_deferred = writer_->put_run_ref(hex, uint32_t(fi->range.start), run, run_len, opt.repair, opt.on_copied);
        if (!out.copy_deferred) defer(hex, *fi, opt.repair);  // the writer's queue was full
      } else if (writer_) {
        if (!writer_->put_run(hex, uint32_t(fi->range.start), run, run_len, opt.repair)) defer(hex, *fi, opt.repair);
      } else
        cache_->put_run(hex, uint32_t(fi->range.start), run, run_len, opt.repair);
    } catch (const Error&) {
    }
  }
  if (!out.ext) land(out, body.data(), body.size(), &body);
  out.local_start = uint32_t(term.range.start - fi->range.start);
  out.local_end = uint32_t(term.range.end - fi->range.start);
  out.source = Source::Cdn;
  return out;
}

void XetBridge::defer(const std::string& hex, const cas::FetchInfo& fi, bool repair) {
  std::lock_guard<std::mutex> g(deferred_mu_);
  deferred_.push_back(Deferred{hex, fi, repair});
}

size_t XetBridge::deferred_count() const {
  std::lock_guard<std::mutex> g(deferred_mu_);
  return deferred_.size();
}

size_t XetBridge::fill_deferred() {
  std::vector<Deferred> todo;
  {
    std::lock_guard<std::mutex> g(deferred_mu_);
    todo.swap(deferred_);
  }
  if (todo.empty() || !cache_ || !cas_) return 0;
  if (writer_) writer_->flush();  // the quarantined runs' promote/discard ops ran first
  std::sort(todo.begin(), todo.end(), [](const Deferred& a, const Deferred& b) {
    return std::tie(a.hex, a.fi.range.start) < std::tie(b.hex, b.fi.range.start);
  });
  size_t done = 0;
  for (size_t i = 0; i < todo.size(); ++i) {
    const Deferred& d = todo[i];
    if (i && d.hex == todo[i - 1].hex && d.fi.range.start == todo[i - 1].fi.range.start) continue;
    if (!d.repair && cache_->find(d.hex, uint32_t(d.fi.range.start), uint32_t(d.fi.range.end))) continue;
    try {
      trace::Span sp("cache", "refill dropped run");
      Bytes body = cas_->fetch(d.fi);
      cache_->put_run(d.hex, uint32_t(d.fi.range.start), body.data(), body.size(), d.repair);
      ++done;
    } catch (const std::exception&) {
      // best effort: a run that cannot be refetched only costs a later miss
    }
  }
  return done;
}

void XetBridge::settle(const std::string& xorb_hex, Source src, uint32_t run_offset, const std::string& pending,
                       bool ok) {
  if (!cache_) return;
  try {
    if (writer_) {  // queued behind the run's own write (same xorb, same writer, FIFO)
      if (src == Source::Peer && !pending.empty()) {
        if (ok) writer_->promote(xorb_hex, run_offset, pending);
        else writer_->discard_pending(pending);
      } else if (src == Source::Cache && !ok) {
        writer_->evict(xorb_hex, run_offset);
      }
      return;
    }
    if (src == Source::Peer && !pending.empty()) {
      if (ok) cache_->promote(xorb_hex, run_offset, pending);
      else cache_->discard_pending(pending);
    } else if (src == Source::Cache && !ok) {
      cache_->evict(xorb_hex, run_offset);
    }
  } catch (const Error&) {
  }
}

void XetBridge::settle(const std::string& xorb_hex, const XorbFetchResult& r, bool ok) {
  settle(xorb_hex, r.source, r.run_offset, r.pending, ok);
}

void XetBridge::print_stats(std::ostream& w) const {
  const uint64_t total = stats_.xorbs_from_cache + stats_.xorbs_from_peer + stats_.xorbs_from_cdn;
  const uint64_t total_bytes = stats_.bytes_from_cache + stats_.bytes_from_peer + stats_.bytes_from_cdn;
  w << "\nXorb fetch stats:\n";
  w << "  Total xorbs:  " << total << "\n";
  w << "  From cache:   " << stats_.xorbs_from_cache.load() << "\n";
  w << "  From peers:   " << stats_.xorbs_from_peer.load() << "\n";
  w << "  From CDN:     " << stats_.xorbs_from_cdn.load() << "\n";
  w << "  Total bytes:  " << total_bytes << "\n";
  if (total_bytes > 0) {
    const double pct = double(stats_.bytes_from_peer.load()) / double(total_bytes) * 100.0;
    w << "  P2P ratio:    " << std::fixed << std::setprecision(1) << pct << "%\n";
  }
  if (stats_.verify_failures.load())
    w << "  Verify fails: " << stats_.verify_failures.load() << " (refetched " << stats_.refetches.load() << ")\n";
}

std::string XetBridge::stats_json() const {
  const uint64_t total_bytes = stats_.bytes_from_cache + stats_.bytes_from_peer + stats_.bytes_from_cdn;
  json::Writer w;
  w.obj();
  w.key("xorbs_from_cache").num_u(stats_.xorbs_from_cache).key("xorbs_from_peer").num_u(stats_.xorbs_from_peer);
  w.key("xorbs_from_cdn").num_u(stats_.xorbs_from_cdn).key("bytes_from_cache").num_u(stats_.bytes_from_cache);
  w.key("bytes_from_peer").num_u(stats_.bytes_from_peer).key("bytes_from_cdn").num_u(stats_.bytes_from_cdn);
  w.key("p2p_ratio").num(total_bytes ? double(stats_.bytes_from_peer) / double(total_bytes) : 0.0, 4);
  w.key("verify_failures").num_u(stats_.verify_failures).key("refetches").num_u(stats_.refetches);
  w.key("peer_bytes").obj();
  if (swarm_)
    for (const auto& [addr, b] : swarm_->peer_bytes()) w.key(addr).num_u(b);
  w.end();
  w.end();
  return w.out();
}

}  // namespace zest
