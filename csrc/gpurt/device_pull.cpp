#include "device_pull.h"

#include <hip/hip_runtime.h>
#include <pthread.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../gpu/zgpu.h"
#include "hip_wait.h"
#include "pinned.h"
#include "bridge.h"
#include "config.h"
#include "storage.h"
#include "swarm.h"
#include "term_jobs.h"
#include "trace.h"
#include "xet_hash.h"
#include "xorb.h"

// Pipeline: batches of terms fill `slots` pinned staging buffers (fetch threads that run on across
// batch boundaries).  A batch's H2D copies (payload + chunk records) go on a copy stream and its
// decode/place/hash kernels on a compute stream, ordered by per-batch events only: batch b's copy
// waits (on the device) for the kernels of batch b - slots, which read the same device staging, and
// a releaser thread hands the host slot back to the fetch workers as soon as batch b's copy landed
// -- no host-side wait for kernels anywhere, so the copy of batch b + 1 overlaps the kernels of
// batch b and PCIe stays busy.  The chunk records come from the header index the fetch workers
// build anyway while validating each run, so the GPU has no header walk to do.

// Flags of the events host threads wait on.  ZEST_EVENT_BLOCKING=1 adds hipEventBlockingSync: a
// waiting thread sleeps in the driver instead of polling (CPU time per pull vs wake-up latency; the
// one-GPU rehearsals share 16 CPUs between all ranks).
static unsigned sync_event_flags() {
  static const unsigned f = [] {
    const char* v = std::getenv("ZEST_EVENT_BLOCKING");
    return unsigned(hipEventDisableTiming) | ((v && v[0] == '1') ? unsigned(hipEventBlockingSync) : 0u);
  }();
  return f;
}

namespace zest::gpurt {

namespace {
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error("HipError", std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  void ensure(size_t count) {
    if (count <= n) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    hip_check(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T) + 4096), "hipMalloc");
    n = count;
  }
};

struct Slot {
  PinnedBuf pin;            // payload staging (fetched runs, back to back)
  uint8_t* host = nullptr;  // = pin.data()
  PinnedBuf rec_pin;        // the batch's chunk records (pinned: the records copy is async too)
  size_t rec_cap = 0;       // records that fit rec_pin
  DevBuf<uint8_t> dev;      // device staging (padded)
  DevBuf<ZgChunk> chunks_dev;
  DevBuf<uint8_t> scratch;  // hash scratch of the batch's ingest launch
  ZgChunk* recs() const { return reinterpret_cast<ZgChunk*>(rec_pin.data()); }
};

size_t env_size(const char* k, size_t dflt) {
  const char* v = std::getenv(k);
  return v && *v ? size_t(std::strtoull(v, nullptr, 10)) : dflt;
}

}  // namespace

// Host side of a pipeline: Xet session, caches, swarm, reconstructions and the settle book.  Shared
// by sibling pipelines (DeviceXetPull::sibling), so a second pipeline costs only its staging.
struct DeviceXetPull::Shared {
  explicit Shared(const DevicePullOptions& o) : cfg(Config::from_env()) {
    {
      trace::Span sp("device", "init: cache scan");
      registry.scan(cfg);
      cache = std::make_unique<storage::XorbCache>(cfg, &registry);
      cache->set_registry_lookup(true);  // a miss needs no cache directory listing on a fetch thread
    }
    if (cfg.cache_writes)  // ZEST_CACHE_WRITE_QUEUE_MB bounds the write-behind queue (0: synchronous)
      if (size_t mb = env_size("ZEST_CACHE_WRITE_QUEUE_MB", 2048)) {
        const size_t bytes = env_size("ZEST_CACHE_WRITE_QUEUE_BYTES", 0);  // (tests: a queue that overflows)
        writer = std::make_unique<storage::CacheWriter>(cache.get(), bytes ? bytes : mb << 20, 2);
      }
    std::vector<net::Addr> boot;
    for (auto& b : o.dht_bootstrap) boot.push_back(net::Addr::parse(b, 6881));
    {
      trace::Span sp("device", "init: swarm");
      swarm = std::make_unique<SwarmDownloader>(cfg, o.tracker, o.p2p, o.dht && o.p2p, boot);
      for (auto& p : o.peers) swarm->add_direct_peer(net::Addr::parse(p, 6881));
    }
    bridge = std::make_unique<XetBridge>(cfg, cache.get(), swarm.get());
    bridge->set_writer(writer.get());
    recs = std::make_unique<ReconCache>(*bridge);
    {
      trace::Span sp("device", "init: xet auth");
      bridge->authenticate(o.repo, o.repo_type, o.revision);
    }
  }
  ~Shared() {
    // runs the write-behind queue dropped are fetched again and cached before the pipeline goes
    // (ZEST_CACHE_REFILL=0: left out); the writer drains first
    try {
      if (writer) writer->flush();
      if (bridge && env_size("ZEST_CACHE_REFILL", 1)) bridge->fill_deferred();
    } catch (...) {
    }
  }
  Config cfg;
  storage::XorbRegistry registry;
  std::unique_ptr<storage::XorbCache> cache;
  std::unique_ptr<storage::CacheWriter> writer;  // destroyed (drained) before the cache
  std::unique_ptr<SwarmDownloader> swarm;
  std::unique_ptr<XetBridge> bridge;
  std::unique_ptr<ReconCache> recs;
  SettleBook book;
};

struct DeviceXetPull::Impl {
  Impl(const DevicePullOptions& o, std::shared_ptr<Shared> shared)
      : sh_(shared ? std::move(shared) : std::make_shared<Shared>(o)),
        device_(o.device),
        cap_(o.staging_bytes),
        threads_(o.threads > 0 ? o.threads : 16),
        nslots_(std::max<size_t>(2, o.slots > 0 ? size_t(o.slots) : env_size("ZEST_DEVICE_SLOTS", 3))) {
    slots_.resize(nslots_);
    if (!o.defer_device) init_device();
  }

  // Device half of the set-up (streams, pinned + device staging): separate from the host half so a
  // caller can run the Xet auth / cache scan while the HIP runtime is still coming up
  // (gpu_worker.cpp).  The pinned slots are page-locked concurrently.  Idempotent.
  void init_device() {
    std::lock_guard<std::mutex> g(init_mu_);
    if (device_ready_) return;
    trace::Span sp("device", "init: staging alloc");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    // The pull's own work (H2D copies, decode/place/hash) is the critical path of a swarm pull: its
    // streams run at the device's greatest priority, the receive-side hashing and the exchanges at
    // normal priority fill what it leaves idle -- the engine's split (zest_amd/engine.py); it
    // matters where ranks share a GPU.  ZEST_PULL_STREAM_PRIORITY=0: normal priority.
    int least = 0, greatest = 0;
    const char* pv = std::getenv("ZEST_PULL_STREAM_PRIORITY");
    if (!(pv && pv[0] == '0') && hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    if (pv && pv[0] == '0') greatest = 0;
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest), "hipStreamCreate");
    hip_check(hipStreamCreateWithPriority(&copy_stream_, hipStreamNonBlocking, greatest), "hipStreamCreate");
    std::vector<std::string> errs(nslots_);
    std::vector<std::thread> pins;
    for (size_t i = 1; i < nslots_; ++i)
      pins.emplace_back([&, i] {
        if (!slots_[i].pin.alloc(cap_ + 4096)) errs[i] = "pinning the staging buffer failed";
      });
    if (!slots_[0].pin.alloc(cap_ + 4096)) errs[0] = "pinning the staging buffer failed";
    for (auto& t : pins) t.join();
    for (auto& e : errs)
      if (!e.empty()) throw Error("HipError", e);
    for (auto& s : slots_) {
      s.host = s.pin.data();
      s.dev.ensure(cap_);
    }
    err_.ensure(1);
    device_ready_ = true;
  }

  ~Impl() {
    s_stop();
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (copy_stream_) (void)hipStreamSynchronize(copy_stream_);
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
    for (hipEvent_t e : timing_events_) (void)hipEventDestroy(e);
    for (auto& s : slots_) {
      s.pin.reset();
      s.rec_pin.reset();
    }
    if (stream_) (void)hipStreamDestroy(stream_);
    if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
  }

  // `n` events for one pass (kept across calls; the previous pass synchronized its streams).
  hipEvent_t* take_events(size_t n) {
    while (events_.size() < n) {
      hipEvent_t e = nullptr;
      hip_check(hipEventCreateWithFlags(&e, sync_event_flags()), "hipEventCreate");
      events_.push_back(e);
    }
    return events_.data();
  }

  // Pull several Xet files (hash, device pointer, size) through ONE pipeline: staging batches
  // cross file boundaries, so there is no per-file drain; every file's Merkle hash is checked in a
  // single kernel launch at the end.
  //
  // Peer runs are quarantined in the disk cache until their file verified; a file that fails
  // (Merkle mismatch, or any device decode error) has its peer runs dropped and its cache runs
  // evicted, then is pulled once more straight from the CDN with the refetched runs replacing the
  // cached ones — so one corrupt copy costs one refetch, not a permanently failing pull.
  std::vector<PullFileStats> pull_files(const std::vector<std::tuple<std::string, uintptr_t, uint64_t>>& files) {
    init_device();
    // HIP's current device is per thread: a caller on any thread (a Python fetch pool, the CLI
    // worker) gets this pipeline's device for the lazy allocations below
    hip_check(hipSetDevice(device_), "hipSetDevice");
    const auto t0 = std::chrono::steady_clock::now();
    const size_t nf = files.size();
    std::vector<const cas::Reconstruction*> recs(nf);
    {
      trace::Span sp("device", "reconstructions");
      std::vector<std::string> errs(nf);
      std::atomic<size_t> k{0};
      auto w = [&]() {
        for (size_t f; (f = k.fetch_add(1)) < nf;) {
          try {
            recs[f] = &sh_->recs->get(std::get<0>(files[f]));
          } catch (const std::exception& e) {
            errs[f] = e.what();
          }
        }
      };
      std::vector<std::thread> ts;
      for (size_t t = 0; t < std::min<size_t>(nf, 8); ++t) ts.emplace_back(w);
      for (auto& t : ts) t.join();
      for (size_t f = 0; f < nf; ++f)
        if (!errs[f].empty()) throw Error("DownloadFailed", std::get<0>(files[f]) + ": " + errs[f]);
    }
    std::vector<size_t> todo(nf);
    for (size_t f = 0; f < nf; ++f) todo[f] = f;
    std::vector<std::string> got(nf);
    std::vector<std::vector<uint32_t>> lens(nf);  // chunk sizes of each file, from its verified attempt
    uint64_t fetched = 0;
    for (int attempt = 0; attempt < 2 && !todo.empty(); ++attempt) {
      FetchOptions opt;
      opt.repair = attempt > 0;
      Attempt at = run_once(files, recs, todo, opt, attempt);
      fetched += at.fetched;
      if (!at.fetch_err.empty()) {
        settle_all(at, recs, todo, [](size_t) { return false; });
        throw Error("DownloadFailed", at.fetch_err);
      }
      // A file is bad only when its own Merkle root misses: the roots are computed from the bytes
      // that landed in HBM, so a decode error in one file (the error word is shared by the batch)
      // cannot pass as good data, and it no longer evicts the cache runs of every other file.
      std::vector<size_t> bad;
      for (size_t j = 0; j < todo.size(); ++j) {
        got[todo[j]] = at.roots[j];
        if (at.roots[j] != std::get<0>(files[todo[j]])) bad.push_back(j);
        else lens[todo[j]] = std::move(at.seg.chunk_lens[j]);
      }
      settle_all(at, recs, todo, [&](size_t j) { return std::find(bad.begin(), bad.end(), j) == bad.end(); });
      if (bad.empty()) {
        todo.clear();
        break;
      }
      if (attempt == 0) sh_->bridge->stats().verify_failures += bad.size();
      else if (at.seg.ingest_err)
        throw Error("IngestError", "code " + std::to_string(at.seg.ingest_err >> 32) + " at " +
                                       std::to_string(at.seg.ingest_err & 0xFFFFFFFFu));
      std::vector<size_t> again;
      for (size_t j : bad) again.push_back(todo[j]);
      if (attempt == 0) sh_->bridge->stats().refetches += again.size();
      todo = std::move(again);
    }
    if (sh_->cfg.cache_max_gb > 0) sh_->cache->trim(uint64_t(sh_->cfg.cache_max_gb * 1e9));  // ZEST_CACHE_MAX_GB
    for (size_t f : todo)
      throw Error("HashMismatch", "device bytes hash " + got[f] + " != " + std::get<0>(files[f]));
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<PullFileStats> out(nf);
    for (size_t f = 0; f < nf; ++f) {
      uint64_t nck = 0;
      for (auto& t : recs[f]->terms) nck += t.range.end - t.range.start;
      out[f].bytes = std::get<2>(files[f]);
      out[f].terms = recs[f]->terms.size();
      out[f].chunks = nck;
      out[f].seconds = secs;
      out[f].fetched_bytes = fetched;  // for the whole call
      out[f].chunk_lens = std::move(lens[f]);
    }
    return out;
  }

  // Term ranges of files into caller memory (the term-sharded swarm pull): every chunk decoded into
  // place and hashed into the caller's table; no Merkle check here (a range is part of a file), so
  // the runs behind the terms stay in book_ until settle(file).  A range whose fetched runs do not
  // match its plan, or any decode error of the call, is refetched once from the CDN.
  std::vector<TermJobResult> pull_terms(const std::vector<TermJob>& jobs, uint8_t* hashes, uint64_t* sizes,
                                        bool repair) {
    init_device();
    hip_check(hipSetDevice(device_), "hipSetDevice");
    std::vector<Seg> segs;
    uint64_t next_chunk = jobs.empty() ? 0 : jobs[0].chunk0;
    for (const TermJob& j : jobs) {
      const cas::Reconstruction& rec = sh_->recs->get(j.xet_hash);
      if (j.t0 > j.t1 || j.t1 > rec.terms.size()) throw Error("RangeOutOfBounds", "term range of " + j.xet_hash);
      if (j.chunk0 != next_chunk) throw Error("InvalidArgument", "term jobs must cover consecutive chunk indices");
      for (uint32_t t = j.t0; t < j.t1; ++t) next_chunk += rec.terms[t].range.end - rec.terms[t].range.start;
      segs.push_back({&rec, j.t0, j.t1, j.dst, j.chunk0});
    }
    std::vector<TermJobResult> out(jobs.size());
    std::vector<size_t> todo(segs.size());
    for (size_t i = 0; i < todo.size(); ++i) todo[i] = i;
    for (int attempt = 0; attempt < 2 && !todo.empty(); ++attempt) {
      FetchOptions opt;
      opt.repair = repair || attempt > 0;
      if (attempt > 0) opt.allow_cache = opt.allow_p2p = false;
      std::vector<Seg> part;
      for (size_t i : todo) part.push_back(segs[i]);
      // a retry covers a subset: its chunk indices are no longer consecutive, so run it seg by seg
      std::vector<std::vector<size_t>> groups;
      if (attempt == 0) groups.push_back(todo);
      else
        for (size_t i : todo) groups.push_back({i});
      std::vector<size_t> bad;
      for (const auto& g : groups) {
        std::vector<Seg> gs;
        for (size_t i : g) gs.push_back(segs[i]);
        SegAttempt at = run_segments(gs, hashes, sizes, opt, attempt, {});
        auto drop = [&](size_t k) {
          for (size_t t = 0; t < at.sources[k].size(); ++t)
            sh_->bridge->settle(gs[k].rec->terms[gs[k].t0 + t].hash_hex, at.sources[k][t].src, at.sources[k][t].run_offset,
                            at.sources[k][t].pending, false);
        };
        if (!at.fetch_err.empty()) {
          // The range is refetched elsewhere: drop the peer runs this call quarantined (never to be
          // Merkle-checked); cache hits and earlier calls' runs wait for their file's verdict.
          for (size_t k = 0; k < gs.size(); ++k)
            for (const TermSource& ts : at.sources[k])
              if (ts.src == Source::Peer && !ts.pending.empty())
                sh_->bridge->settle(std::string(), ts.src, ts.run_offset, ts.pending, false);
          throw Error("DownloadFailed", at.fetch_err);
        }
        for (size_t k = 0; k < gs.size(); ++k) {
          const size_t i = g[k];
          if (at.ingest_err || !at.planned_ok[k]) {
            drop(k);
            bad.push_back(i);
            continue;
          }
          TermJobResult& r = out[i];
          r.chunk_lens = std::move(at.chunk_lens[k]);
          r.fetched += at.seg_fetched[k];
          for (size_t t = 0; t < at.sources[k].size(); ++t) {
            const TermSource& ts = at.sources[k][t];
            const cas::Term& term = gs[k].rec->terms[gs[k].t0 + t];
            sh_->book.add(jobs[i].xet_hash, term.hash_hex, ts.src, ts.run_offset, ts.pending);
            (ts.src == Source::Peer ? r.from_peer : ts.src == Source::Cache ? r.from_cache : r.from_cdn) +=
                term.unpacked_length;
          }
        }
        if (at.ingest_err && attempt > 0)
          throw Error("IngestError", "code " + std::to_string(at.ingest_err >> 32) + " at " +
                                         std::to_string(at.ingest_err & 0xFFFFFFFFu));
      }
      if (!bad.empty() && attempt == 0) sh_->bridge->stats().refetches += bad.size();
      todo = std::move(bad);
    }
    if (!todo.empty()) throw Error("IngestError", "term range of " + jobs[todo[0]].xet_hash + " does not match its plan");
    return out;
  }

  // Order everything this pipeline queues from now on after `ev` (a caller's event, e.g. the zero-fill
  // of the tables its kernels write): only the compute stream writes caller memory.
  void order_after(hipEvent_t ev) {
    init_device();
    hip_check(hipStreamWaitEvent(stream_, ev, 0), "hipStreamWaitEvent (order_after)");
  }

  size_t settle(const std::string& hex, bool ok) { return sh_->book.settle(*sh_->bridge, hex, ok); }
  void flush_cache_writes() {
    if (sh_->writer) sh_->writer->flush();
    sh_->bridge->fill_deferred();  // runs the full write-behind queue dropped: refetched and cached now
  }
  std::vector<TermShape> term_shapes(const std::string& hex) { return sh_->recs->shapes(hex); }

  std::string stats_json() const { return sh_->bridge->stats_json(); }

  size_t staging_bytes() const { return cap_; }

  PullProgressFn progress_;  // set for the duration of one pull_files call

  struct TermSource {
    Source src = Source::Cdn;
    uint32_t run_offset = 0;
    std::string pending;  // quarantine file of a peer run (empty: none)
  };
  // A contiguous term range of one file: outputs from device address `dst`, chunk hashes / sizes
  // at index chunk0.. of the caller's tables.
  struct Seg {
    const cas::Reconstruction* rec;
    uint32_t t0, t1;
    uintptr_t dst;
    uint64_t chunk0;
  };
  struct SegAttempt {
    std::vector<std::vector<TermSource>> sources;   // per seg, per term
    std::vector<std::vector<uint32_t>> chunk_lens;  // per seg: uncompressed chunk sizes
    std::vector<uint8_t> planned_ok;                // per seg: every fetched run matched the plan
    std::vector<uint64_t> seg_fetched;              // per seg: bytes moved
    unsigned long long ingest_err = 0;
    std::string fetch_err;
    uint64_t fetched = 0;
  };
  struct Attempt {
    SegAttempt seg;                  // one seg per file of the attempt
    std::vector<std::string> roots;  // per file of the attempt: Merkle root (Xet hex)
    uint64_t fetched = 0;
    std::string fetch_err;
  };

  // A term of a pass in segment order: its segment, term index, output offset from the pass's base
  // address, first chunk (pass-relative), chunk count and unpacked size.
  struct GTerm {
    size_t seg, term;
    uint64_t dst;
    uint64_t chunk;
    uint32_t nchunks;
    uint64_t ulen;
  };
  struct TermFetch {
    uint64_t src_at = 0, len = 0;  // the run's chunk span in the slot: offset, bytes
    TermSource src;
    bool planned = true;           // the run matched the term's plan (else its records stay zero)
  };
  // One term of a pass: fetch its run through the cache -> P2P -> CDN waterfall into `region` (the
  // term's reserved part of a pinned staging slot, `room` bytes, at `region_off` in the slot) and
  // write its chunks' device records into `cr` and their sizes into `lens`.  A run that does not
  // match the plan keeps zero (no-op) records, so its file fails the Merkle check and takes the
  // repair path.  `copied` runs once no writer copy thread reads the region any more (now, unless
  // the fetch deferred the cache copy to the writer).  Throws on a fetch error.
  TermFetch fetch_term_into(const cas::Reconstruction& rec, const GTerm& g, const FetchOptions& topt,
                            const std::function<void()>& copied, uint8_t* region, uint64_t room, uint64_t region_off,
                            uint32_t tag, ZgChunk* cr, uint32_t* lens, TermSource& src_out) {
    auto sink = [&](size_t nbytes) -> uint8_t* { return nbytes <= room ? region : nullptr; };
    XorbFetchResult r;
    try {
      r = sh_->bridge->fetch_term(rec.terms[g.term], rec, topt, sink);
    } catch (...) {
      copied();
      throw;
    }
    if (!r.copy_deferred) copied();
    TermFetch tf;
    tf.src = TermSource{r.source, r.run_offset, r.pending};
    src_out = tf.src;  // (recorded before any check below throws: a quarantined run is dropped on failure)
    auto idx = xet::index_chunks(r.bytes(), r.size());
    if (r.local_end > idx.size() || r.local_start >= r.local_end)
      throw Error("RangeOutOfBounds", rec.terms[g.term].hash_hex);
    const uint64_t a = idx[r.local_start].header_off;
    const uint64_t e_end = idx[r.local_end - 1].header_off + xet::kChunkHeaderLen + idx[r.local_end - 1].clen;
    if (r.ext) {
      tf.src_at = region_off + a;  // already in place
    } else {
      if (e_end - a > room) throw Error("TermTooLarge", "term " + std::to_string(g.term) + " exceeds its bound");
      std::memcpy(region, r.data.data() + a, e_end - a);
      tf.src_at = region_off;
    }
    tf.len = e_end - a;
    const uint64_t run0 = tf.src_at;
    uint64_t uoff = 0;
    bool ok = r.local_end - r.local_start == g.nchunks;
    for (uint32_t c = r.local_start; ok && c < r.local_end; ++c) {
      const xet::ChunkEntry& e = idx[c];
      const uint32_t sc = uint32_t(e.scheme);
      if (sc > 2 || (sc == 0 && e.clen != e.ulen) || e.ulen > 128u * 1024u) {
        ok = false;
        break;
      }
      cr[c - r.local_start] = ZgChunk{run0 + (e.header_off - a) + xet::kChunkHeaderLen, g.dst + uoff, e.clen, e.ulen, sc, tag};
      lens[c - r.local_start] = e.ulen;
      uoff += e.ulen;
    }
    if (!ok || uoff != g.ulen) {
      std::fill(cr, cr + g.nchunks, ZgChunk{});
      tf.planned = false;
    }
    return tf;
  }

  // Publish (ok) or drop/evict (!ok) the cache runs behind every term of the attempt's files.
  template <typename OkFn>
  void settle_all(const Attempt& at, const std::vector<const cas::Reconstruction*>& recs,
                  const std::vector<size_t>& todo, OkFn ok) {
    for (size_t j = 0; j < todo.size(); ++j) {
      const auto& rec = *recs[todo[j]];
      const bool good = ok(j);
      for (size_t i = 0; i < at.seg.sources[j].size() && i < rec.terms.size(); ++i) {
        const TermSource& ts = at.seg.sources[j][i];
        sh_->bridge->settle(rec.terms[i].hash_hex, ts.src, ts.run_offset, ts.pending, good);
      }
    }
  }

  // Whole files[todo] through run_segments into the internal hash table, then one Merkle launch.
  Attempt run_once(const std::vector<std::tuple<std::string, uintptr_t, uint64_t>>& all_files,
                   const std::vector<const cas::Reconstruction*>& all_recs, const std::vector<size_t>& todo,
                   const FetchOptions& opt, int attempt) {
    const size_t nf = todo.size();
    Attempt at;
    std::vector<Seg> segs;
    std::vector<uint64_t> file_chunk0(nf + 1, 0);
    for (size_t f = 0; f < nf; ++f) {
      const auto& fl = all_files[todo[f]];
      const cas::Reconstruction& rec = *all_recs[todo[f]];
      uint64_t off = 0, c = 0;
      for (const auto& t : rec.terms) {
        off += t.unpacked_length;
        c += t.range.end - t.range.start;
      }
      if (off != std::get<2>(fl)) throw Error("SizeMismatch", std::get<0>(fl) + " is " + std::to_string(off) + " bytes");
      segs.push_back({&rec, 0, uint32_t(rec.terms.size()), std::get<1>(fl), file_chunk0[f]});
      file_chunk0[f + 1] = file_chunk0[f] + c;
    }
    const uint64_t nck = file_chunk0[nf];
    hashes_.ensure(nck ? nck * 32 : 32);
    sizes_.ensure(nck ? nck : 1);
    std::function<void(size_t, uint64_t)> prog;
    if (progress_) prog = [&](size_t seg, uint64_t bytes) { progress_(todo[seg], attempt, bytes); };
    at.seg = run_segments(segs, hashes_.p, sizes_.p, opt, attempt, prog);
    at.fetched = at.seg.fetched;
    at.fetch_err = at.seg.fetch_err;
    if (!at.fetch_err.empty()) return at;
    // Merkle roots of every file in one launch
    trace::Span merkle_span("device", "merkle verify");
    std::vector<ZgMerkleJob> mjobs(nf);
    uint64_t max_leaves = 1;
    for (size_t f = 0; f < nf; ++f) {
      mjobs[f] = ZgMerkleJob{file_chunk0[f], file_chunk0[f + 1] - file_chunk0[f], 1, 0};
      max_leaves = std::max<uint64_t>(max_leaves, mjobs[f].n_leaves);
    }
    std::vector<uint8_t> roots(32 * std::max<size_t>(nf, 1));
    if (nf) {
      merkle_job_.ensure(nf);
      hip_check(hipMemcpyAsync(merkle_job_.p, mjobs.data(), sizeof(ZgMerkleJob) * nf, hipMemcpyHostToDevice, stream_),
                "job H2D");
      const size_t sb = zg_merkle_scratch_bytes(max_leaves, int(nf));
      merkle_scratch_.ensure(sb);
      root_.ensure(32 * nf);
      hip_check(zg_merkle(hashes_.p, sizes_.p, merkle_job_.p, int(nf), root_.p, merkle_scratch_.p, sb, stream_),
                "merkle");
      hip_check(hipMemcpyAsync(roots.data(), root_.p, 32 * nf, hipMemcpyDeviceToHost, stream_), "root D2H");
      hip_check(gpu::idle_stream_sync(stream_), "sync");
    }
    for (size_t f = 0; f < nf; ++f) {
      xet::Hash h;
      std::memcpy(h.data(), roots.data() + 32 * f, 32);
      at.roots.push_back(xet::to_hex(h));
    }
    return at;
  }

  // One pass over segments: fetch (+ chunk records) -> staging -> H2D -> place/hash.  Segments must
  // cover consecutive chunk indices (chunk0 of seg k+1 = chunk0 of seg k + its chunks): hashes and
  // sizes of the pass go to hashes[segs[0].chunk0 ..] in one run.
  SegAttempt run_segments(const std::vector<Seg>& segs, uint8_t* hash_out, uint64_t* size_out, const FetchOptions& opt,
                          int attempt, const std::function<void(size_t, uint64_t)>& progress) {
    (void)attempt;
    s_drain();  // the streaming engine shares the slots and streams: nothing of it may be in flight
    const size_t ns = segs.size();
    SegAttempt at;
    at.sources.resize(ns);
    at.chunk_lens.resize(ns);
    at.planned_ok.assign(ns, 1);
    at.seg_fetched.assign(ns, 0);
    // Global term list in segment order; chunk indices are relative to segs[0].chunk0.
    std::vector<GTerm> gt;
    std::vector<uint64_t> seg_chunk0(ns + 1, 0), seg_dst0(ns, 0);
    uintptr_t base = UINTPTR_MAX, top_addr = 0;
    const uint64_t hash_base = ns ? segs[0].chunk0 : 0;
    for (size_t s = 0; s < ns; ++s) {
      uint64_t bytes = 0;
      for (uint32_t t = segs[s].t0; t < segs[s].t1; ++t) bytes += segs[s].rec->terms[t].unpacked_length;
      base = std::min(base, segs[s].dst);
      top_addr = std::max<uintptr_t>(top_addr, segs[s].dst + bytes);
    }
    for (size_t s = 0; s < ns; ++s) {
      const Seg& sg = segs[s];
      if (sg.chunk0 != hash_base + seg_chunk0[s]) throw Error("InvalidArgument", "segments must cover consecutive chunks");
      at.sources[s].resize(sg.t1 - sg.t0);
      seg_dst0[s] = sg.dst - base;
      uint64_t off = 0, c = seg_chunk0[s];
      for (uint32_t i = sg.t0; i < sg.t1; ++i) {
        const auto& t = sg.rec->terms[i];
        const uint32_t n = uint32_t(t.range.end - t.range.start);
        gt.push_back({s, i, sg.dst - base + off, c, n, t.unpacked_length});
        off += t.unpacked_length;
        c += n;
      }
      seg_chunk0[s + 1] = c;
      at.chunk_lens[s].assign(size_t(c - seg_chunk0[s]), 0);
    }
    const uint64_t nck = seg_chunk0[ns];
    const size_t n = gt.size();
    uint8_t* dst = ns ? reinterpret_cast<uint8_t*>(base) : nullptr;
    const uint64_t dst_size = ns ? uint64_t(top_addr - base) : 0;
    hip_check(hipMemsetAsync(err_.p, 0, sizeof(unsigned long long), stream_), "hipMemset");
    std::string& fetch_err = at.fetch_err;
    {
      // Batches: consecutive terms whose fetched-size bounds fit one staging slot, so every term
      // has a reserved region of the pinned buffer (no refetch, no second copy pass: workers
      // receive / copy their run straight into place).  Batch b fills slot b % slots.
      uint64_t max_bound = 0;
      for (size_t i = 0; i < n; ++i) max_bound = std::max(max_bound, term_bound(gt[i].ulen, gt[i].nchunks));
      if (max_bound > cap_) grow_staging(max_bound);  // one huge term: enlarge every slot
      struct Batch {
        size_t begin = 0, end = 0;
        std::vector<uint64_t> off, len, src_at;  // per term: region, fetched bytes, run start
      };
      std::vector<Batch> batches;
      std::vector<uint32_t> batch_of(n);
      for (size_t next = 0; next < n;) {
        Batch bt;
        bt.begin = next;
        uint64_t pos = 0;
        size_t end = next;
        // the pass's first batch is small (ZEST_FIRST_BATCH_MB, 128): nothing overlaps its fetch, so
        // the copy engine starts after ~128 MiB has arrived instead of a whole slot
        const uint64_t cap_b = batches.empty() ? first_batch_cap() : cap_;
        while (end < n) {
          const uint64_t bound = term_bound(gt[end].ulen, gt[end].nchunks);
          if (pos + bound > cap_b && end > next) break;
          bt.off.push_back(pos);
          pos += bound;
          batch_of[end++] = uint32_t(batches.size());
        }
        bt.end = end;
        bt.len.assign(end - next, 0);
        bt.src_at.assign(end - next, 0);
        batches.push_back(std::move(bt));
        next = end;
      }
      const size_t nb = batches.size();
      const size_t S = nslots_;
      auto chunk_lo = [&](size_t b) { return gt[batches[b].begin].chunk; };
      auto chunk_hi = [&](size_t b) { return batches[b].end < n ? gt[batches[b].end].chunk : nck; };
      // every slot's pinned record table holds the largest batch (the streams are idle here: the
      // previous pass synchronized them)
      size_t max_recs = 1;
      for (size_t b = 0; b < nb; ++b) max_recs = std::max<size_t>(max_recs, size_t(chunk_hi(b) - chunk_lo(b)));
      for (auto& sl : slots_)
        if (sl.rec_cap < max_recs) {
          const size_t cap = std::max(max_recs, size_t(16384));
          if (!sl.rec_pin.alloc(cap * sizeof(ZgChunk))) throw Error("HipError", "pinning the chunk records failed");
          sl.rec_cap = cap;
        }
      hipEvent_t* ev = take_events(2 * nb);  // ev[2b]: batch b's copies landed; ev[2b+1]: its kernels ran
      // ZEST_DEVICE_TIMING=1: timed events around every batch's copy and kernels (device timeline
      // of the pass: copy / kernel busy time and how much of it overlapped, timeline_json())
      hipEvent_t* tev = timing_ ? take_timing_events(4 * nb) : nullptr;
      // Continuous pipeline: the fetch workers take terms in order across batch boundaries, so the
      // next batches' terms are already in flight while the current batch's slowest transfers finish
      // (a per-batch join left the connections ~45 % idle: tools/direct_bench.py under ZEST_TRACE).
      // A worker may fill slot b % S for batch b once ready[b % S] >= b, i.e. once the H2D copy of
      // batch b - S out of that slot has completed (the releaser thread watches the copy events);
      // the submitting thread (this one) waits for each batch's last term and queues its copies and
      // kernels without waiting for the GPU.
      std::mutex mu;
      std::condition_variable cv;
      std::vector<size_t> ready(S);
      for (size_t i = 0; i < S; ++i) ready[i] = i;
      std::vector<size_t> remaining(nb);
      for (size_t b = 0; b < nb; ++b) remaining[b] = batches[b].end - batches[b].begin;
      // Cache copies of runs still reading batch b's host slot: the write-behind writer's copy
      // threads take them (FetchOptions::on_copied), so the fetch threads never copy a run for the
      // cache; the slot goes back to the workers only when its H2D landed AND these are done.
      std::vector<size_t> copies(nb, 0);
      auto copies_done = [&]() {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return std::all_of(copies.begin(), copies.end(), [](size_t c) { return c == 0; }); });
      };
      bool abort = false;
      uint64_t h2d_bytes = 0;  // payload bytes queued for H2D this pass (timeline)
      std::atomic<size_t> k{0};
      auto fail = [&](const std::string& what) {
        std::lock_guard<std::mutex> g(mu);
        if (fetch_err.empty()) fetch_err = what;
        abort = true;
        cv.notify_all();
      };
      auto worker = [&]() {
        pthread_setname_np(pthread_self(), "zest-fetch");
        while (true) {
          const size_t i = k.fetch_add(1);
          if (i >= n) return;
          const size_t b = batch_of[i];
          Batch& bt = batches[b];
          Slot& s = slots_[b % S];
          {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return abort || ready[b % S] >= b; });
            if (abort) return;
          }
          const size_t j = i - bt.begin;
          try {
            const cas::Reconstruction& rec = *segs[gt[i].seg].rec;
            // The run is received straight into this term's region of the pinned buffer when it
            // fits (no intermediate heap buffer); otherwise only its chunk span is copied in.
            uint8_t* region = s.host + bt.off[j];
            const uint64_t room = (i + 1 < bt.end ? bt.off[j + 1] : cap_) - bt.off[j];
            FetchOptions topt = opt;
            {
              std::lock_guard<std::mutex> g(mu);
              ++copies[b];
            }
            auto copied = [&mu, &cv, &copies, b]() {
              {
                std::lock_guard<std::mutex> g(mu);
                --copies[b];
              }
              cv.notify_all();
            };
            if (sh_->writer) topt.on_copied = copied;
            ZgChunk* cr = s.recs() + (gt[i].chunk - chunk_lo(b));
            uint32_t* lens = at.chunk_lens[gt[i].seg].data() + (gt[i].chunk - seg_chunk0[gt[i].seg]);
            const TermFetch tf = fetch_term_into(rec, gt[i], topt, copied, region, room, bt.off[j], uint32_t(j), cr, lens,
                                                 at.sources[gt[i].seg][gt[i].term - segs[gt[i].seg].t0]);
            bt.src_at[j] = tf.src_at;
            bt.len[j] = tf.len;
            if (!tf.planned) {
              std::lock_guard<std::mutex> g(mu);
              at.planned_ok[gt[i].seg] = 0;
            }
          } catch (const std::exception& e) {
            fail(e.what());
            return;
          }
          std::lock_guard<std::mutex> g(mu);
          if (--remaining[b] == 0) cv.notify_all();
        }
      };
      // Releaser: batch b's host slot goes back to the workers once its copies landed; with a
      // progress callback, the batch's bytes are reported once its kernels ran.  Events are per
      // batch, so nothing is re-recorded under its feet.
      std::deque<size_t> issued;  // batches queued on the GPU, in order; SIZE_MAX ends the thread
      auto releaser = [&]() {
        pthread_setname_np(pthread_self(), "zest-release");
        (void)hipSetDevice(device_);
        while (true) {
          size_t b;
          {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return !issued.empty(); });
            b = issued.front();
            issued.pop_front();
          }
          if (b == SIZE_MAX) return;
          const bool copied = gpu::idle_event_sync(ev[2 * b]) == hipSuccess;
          {
            std::unique_lock<std::mutex> g(mu);
            if (!copied) {
              if (fetch_err.empty()) fetch_err = "hipEventSynchronize (H2D)";
              abort = true;
            }
            cv.wait(g, [&] { return copies[b] == 0; });  // the writer's copy threads are done with the slot
            ready[b % S] = b + S;
            cv.notify_all();
          }
          if (progress && copied && gpu::idle_event_sync(ev[2 * b + 1]) == hipSuccess) {
            // batches run in term order, and terms are in segment order: each touched segment's
            // bytes are complete up to the end of its last term in this batch
            const Batch& bt = batches[b];
            for (size_t i = bt.begin; i < bt.end; ++i)
              if (i + 1 == bt.end || gt[i + 1].seg != gt[i].seg)
                progress(gt[i].seg, gt[i].dst + gt[i].ulen - seg_dst0[gt[i].seg]);
          }
        }
      };
      std::vector<std::thread> ts;
      const int nt = int(std::min<size_t>(size_t(threads_), n));
      for (int t = 0; t < nt; ++t) ts.emplace_back(worker);
      std::thread rel(releaser);
      auto stop_releaser = [&]() {
        {
          std::lock_guard<std::mutex> g(mu);
          issued.push_back(SIZE_MAX);
        }
        cv.notify_all();
        rel.join();
      };
      try {
        for (size_t b = 0; b < nb; ++b) {
          {
            trace::Span sp("device", "wait fetch batch");
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return abort || remaining[b] == 0; });
            if (abort) break;
          }
          const Batch& bt = batches[b];
          Slot& s = slots_[b % S];
          uint64_t top = 0;
          for (size_t j = 0; j < bt.len.size(); ++j) {
            at.fetched += bt.len[j];
            at.seg_fetched[gt[bt.begin + j].seg] += bt.len[j];
            top = std::max<uint64_t>(top, bt.src_at[j] + bt.len[j]);
          }
          const uint64_t c0 = chunk_lo(b);
          const int nchunks = int(chunk_hi(b) - c0);
          uint64_t ubytes = 0;
          for (size_t i = bt.begin; i < bt.end; ++i) ubytes += gt[i].ulen;
          bool compressed = false;
          for (int c = 0; c < nchunks && !compressed; ++c) compressed = s.recs()[c].scheme != 0;
          const size_t hs_bytes = zg_ingest_scratch_bytes(nchunks, ubytes);
          // the slot's device staging, records and scratch are read by batch b - S's kernels
          if (b >= S && (s.chunks_dev.n < size_t(nchunks ? nchunks : 1) || s.scratch.n < hs_bytes))
            hip_check(gpu::idle_event_sync(ev[2 * (b - S) + 1]), "hipEventSynchronize");  // growing: wait, then free
          s.chunks_dev.ensure(size_t(nchunks ? nchunks : 1));
          s.scratch.ensure(hs_bytes);
          trace::Span submit_span("device", "queue H2D + place/hash");
          submit_span.arg("\"terms\":" + std::to_string(bt.end - bt.begin) + ",\"bytes\":" + std::to_string(top));
          if (b >= S) hip_check(hipStreamWaitEvent(copy_stream_, ev[2 * (b - S) + 1], 0), "hipStreamWaitEvent");
          if (tev) hip_check(hipEventRecord(tev[4 * b], copy_stream_), "event");
          // Only the fetched bytes cross PCIe: each term owns a region sized for its worst case
          // (term_bound: every chunk stored raw), and a compressed run fills ~88 % of it on bf16
          // weights, so one copy of [0, top) moved the holes too (70B bf16 public path: 141 GB over
          // PCIe for 123.6 GB of runs, 55.2 GB/s against the engine's 64.3).  Runs are copied to
          // the same offsets (the chunk records address the slot).
          // (ZEST_H2D_WHOLE_SPAN=1: the old single copy of [0, top), for A/B runs)
          static const bool whole_span = env_size("ZEST_H2D_WHOLE_SPAN", 0) != 0;
          // Neighbours merge across gaps of at most 64 KiB (ZEST_H2D_MERGE_GAP): small terms share a
          // copy, while a 64 MiB term's ~0.6 MB of worst-case slack stays off PCIe -- with 1 MiB
          // the random-bytes 70B pull moved 142.3 GB for 141.1 (public path 54.2 vs 54.8 GB/s with
          // no merging, same box; the per-term copies cost nothing visible: 56.3 GB/s busy).
          static const uint64_t merge_gap = env_size("ZEST_H2D_MERGE_GAP", size_t(64) << 10);
          const auto ranges = whole_span ? std::vector<std::pair<uint64_t, uint64_t>>{{0, top}}
                                         : copy_ranges(bt.src_at, bt.len, merge_gap);
          for (const auto& [lo, hi] : ranges) {
            hip_check(hipMemcpyAsync(s.dev.p + lo, s.host + lo, hi - lo, hipMemcpyHostToDevice, copy_stream_), "H2D");
            h2d_bytes += hi - lo;
          }
          if (nchunks)
            hip_check(hipMemcpyAsync(s.chunks_dev.p, s.recs(), sizeof(ZgChunk) * size_t(nchunks), hipMemcpyHostToDevice,
                                     copy_stream_),
                      "H2D chunk records");
          hip_check(hipEventRecord(ev[2 * b], copy_stream_), "event");
          if (tev) hip_check(hipEventRecord(tev[4 * b + 1], copy_stream_), "event");
          hip_check(hipStreamWaitEvent(stream_, ev[2 * b], 0), "hipStreamWaitEvent");
          if (tev) hip_check(hipEventRecord(tev[4 * b + 2], stream_), "event");
          // decode (when the batch has compressed chunks) + one fused pass placing raw chunks and
          // hashing every chunk (csrc/gpu/blake3_flat.hip PlaceSrc)
          hip_check(zg_ingest_chunks(s.dev.p, top, dst, dst_size, s.chunks_dev.p, nchunks, compressed ? 1 : 0, err_.p,
                                     hash_out + 32 * (hash_base + c0), size_out ? size_out + hash_base + c0 : nullptr, 0,
                                     s.scratch.p, hs_bytes, stream_),
                    "ingest");
          hip_check(hipEventRecord(ev[2 * b + 1], stream_), "event");
          if (tev) hip_check(hipEventRecord(tev[4 * b + 3], stream_), "event");
          {
            std::lock_guard<std::mutex> g(mu);
            issued.push_back(b);
          }
          cv.notify_all();
        }
      } catch (const std::exception& e) {
        fail(e.what());
        for (auto& t : ts) t.join();
        (void)hipStreamSynchronize(copy_stream_);
        (void)hipStreamSynchronize(stream_);
        stop_releaser();
        copies_done();  // no copy thread may still read the slots (or these counters) after return
        throw;
      }
      for (auto& t : ts) t.join();
      copies_done();
      const hipError_t e1 = gpu::idle_stream_sync(copy_stream_);
      const hipError_t e2 = gpu::idle_stream_sync(stream_);
      stop_releaser();
      hip_check(e1, "sync copy stream");
      hip_check(e2, "sync compute stream");
      if (tev && nb) record_timeline(tev, nb, h2d_bytes);
    }
    if (!fetch_err.empty()) return at;
    hip_check(hipMemcpy(&at.ingest_err, err_.p, sizeof at.ingest_err, hipMemcpyDeviceToHost), "err D2H");
    return at;
  }


  // ---------------------------------------------------------------------------------------------
  // Streaming submission (the swarm pull's rounds at N > 1).  pull_terms() is one pass that drains
  // its streams before it returns, so a caller issuing one call per round serialized every round
  // boundary.  submit_terms() instead appends an item -- one round's term
  // ranges -- to ONE continuous pipeline whose fetch workers, submitter and releaser threads, pinned
  // slots and copy / compute streams persist across items: the workers take terms in submission
  // order across item boundaries, the submitter queues every staging batch's H2D copy and
  // decode/place/hash kernels as soon as its terms are in, and the releaser hands a host slot back
  // once its copy landed.  Nothing waits for the GPU between items.  wait_item(ticket) returns once
  // the item's last kernels are queued, with a HIP event that completes with them; the caller
  // orders the item's exchange after that event (stream wait, or a peer ready counter) without ever
  // blocking on the device.  Batches never cross items, and a failed item (a fetch that fails from
  // every source, or a run that does not match its plan) skips its remaining fetches and GPU work,
  // so the caller can hand it to another rank.  Device decode errors are reported per item by
  // item_error() (an error word per item, copied back behind its kernels).
  struct SItem {
    uint64_t ticket = 0;
    std::vector<TermJob> jobs;
    std::vector<Seg> segs;
    std::vector<GTerm> gt;
    std::vector<uint64_t> seg_chunk0;
    uint8_t* dst = nullptr;  // base device address (the item's lowest output byte)
    uint64_t dst_size = 0;
    uint8_t* hash_out = nullptr;  // hashes + 32 * chunk0 of the item
    uint64_t* size_out = nullptr;
    SegAttempt at;
    size_t b0 = 0, nb = 0;  // global batches [b0, b0 + nb)
    bool failed = false;
    std::string err;
    bool queued = false;     // the submitter passed the item's last batch (done event recorded)
    bool collected = false;  // wait_item() ran
    hipEvent_t done = nullptr;
    size_t eslot = 0;        // error word index
  };
  struct SBatch {
    SItem* item = nullptr;
    size_t begin = 0, end = 0;  // terms [begin, end) of item->gt
    std::vector<uint64_t> off, len, src_at;
    uint64_t c_lo = 0, c_hi = 0;  // item-relative chunk range
    size_t remaining = 0;
    size_t copies = 0;
    bool gpu = false;  // its H2D + kernels were queued
    uint64_t h2d = 0;  // bytes copied
    std::array<hipEvent_t, 4> tev{};  // ZEST_DEVICE_TIMING: copy start / end, kernels start / end
  };
  static constexpr size_t kErrRing = 4096;

  void s_start() {
    if (s_started_) return;
    init_device();
    hip_check(hipSetDevice(device_), "hipSetDevice");
    const size_t S = nslots_;
    sh2d_.assign(S, nullptr);
    skern_.assign(S, nullptr);
    skern_set_.assign(S, 0);
    sready_.resize(S);
    for (size_t i = 0; i < S; ++i) {
      hip_check(hipEventCreateWithFlags(&sh2d_[i], sync_event_flags()), "hipEventCreate");
      hip_check(hipEventCreateWithFlags(&skern_[i], sync_event_flags()), "hipEventCreate");
      sready_[i] = i;
    }
    serr_.ensure(kErrRing);
    if (!serr_host_.alloc(kErrRing * sizeof(unsigned long long))) throw Error("HipError", "pinning the error words failed");
    std::memset(serr_host_.data(), 0, kErrRing * sizeof(unsigned long long));
    const int nt = threads_ > 0 ? threads_ : 16;
    for (int t = 0; t < nt; ++t) sworkers_.emplace_back([this] { s_worker(); });
    ssubmitter_ = std::thread([this] { s_submitter(); });
    sreleaser_ = std::thread([this] { s_releaser(); });
    s_started_ = true;
  }

  void s_stop() {
    if (!s_started_) return;
    {
      std::lock_guard<std::mutex> g(smu_);
      sstop_ = true;
    }
    scv_.notify_all();
    for (auto& t : sworkers_) t.join();
    ssubmitter_.join();
    sreleaser_.join();
    sworkers_.clear();
    (void)hipStreamSynchronize(copy_stream_);
    (void)hipStreamSynchronize(stream_);
    for (auto& it : sitems_)
      if (it->done) (void)hipEventDestroy(it->done);
    sitems_.clear();
    for (hipEvent_t e : sh2d_) (void)hipEventDestroy(e);
    for (hipEvent_t e : skern_) (void)hipEventDestroy(e);
    sh2d_.clear();
    skern_.clear();
    s_started_ = false;
  }

  // Every submitted batch released (fetched, queued, copy landed, slot back) and both streams idle.
  void s_drain() {
    if (!s_started_) return;
    {
      std::unique_lock<std::mutex> g(smu_);
      scv_.wait(g, [&] { return sreleased_ == sbatch_total_; });
    }
    hip_check(gpu::idle_stream_sync(copy_stream_), "sync copy stream");
    hip_check(gpu::idle_stream_sync(stream_), "sync compute stream");
  }

  // Forget every item (their events too): between pulls, once the caller waited for all of them.
  // `cancel`: items still fetching are marked failed first, so their remaining terms are skipped.
  void s_reset(bool cancel) {
    if (!s_started_) return;
    if (cancel) {
      {
        std::lock_guard<std::mutex> g(smu_);
        for (auto& it : sitems_)
          if (!it->queued && !it->failed) {
            it->failed = true;
            it->err = "cancelled";
          }
      }
      scv_.notify_all();
    }
    s_drain();
    std::lock_guard<std::mutex> g(smu_);
    if (timing_) {  // the streamed pass's device timeline (timeline_json), then its events go
      std::vector<std::array<hipEvent_t, 4>> tev;
      uint64_t h2d = 0;
      for (auto& b : sbatches_)
        if (b.gpu && b.tev[0]) {
          tev.push_back(b.tev);
          h2d += b.h2d;
        }
      record_timeline(tev, h2d);
      for (auto& b : sbatches_)
        for (auto& e : b.tev)
          if (e) (void)hipEventDestroy(e);
    }
    for (auto& it : sitems_)
      if (it->done) (void)hipEventDestroy(it->done);
    sitems_.clear();
    sbatches_.clear();
    swork_.clear();
    swork_next_ = 0;
    sb0_ = sbatch_total_;
  }

  SItem* s_find(uint64_t ticket) {
    for (auto& it : sitems_)
      if (it->ticket == ticket) return it.get();
    throw Error("InvalidArgument", "unknown pull ticket " + std::to_string(ticket));
  }

  uint64_t submit_terms(const std::vector<TermJob>& jobs, uint8_t* hashes, uint64_t* sizes) {
    s_start();
    auto item = std::make_unique<SItem>();
    SItem& it = *item;
    it.jobs = jobs;
    uint64_t next_chunk = jobs.empty() ? 0 : jobs[0].chunk0;
    for (const TermJob& j : jobs) {
      const cas::Reconstruction& rec = sh_->recs->get(j.xet_hash);
      if (j.t0 > j.t1 || j.t1 > rec.terms.size()) throw Error("RangeOutOfBounds", "term range of " + j.xet_hash);
      if (j.chunk0 != next_chunk) throw Error("InvalidArgument", "term jobs must cover consecutive chunk indices");
      for (uint32_t t = j.t0; t < j.t1; ++t) next_chunk += rec.terms[t].range.end - rec.terms[t].range.start;
      it.segs.push_back({&rec, j.t0, j.t1, j.dst, j.chunk0});
    }
    const size_t ns = it.segs.size();
    it.at.sources.resize(ns);
    it.at.chunk_lens.resize(ns);
    it.at.planned_ok.assign(ns, 1);
    it.at.seg_fetched.assign(ns, 0);
    uintptr_t base = UINTPTR_MAX, top_addr = 0;
    for (const Seg& sg : it.segs) {
      uint64_t bytes = 0;
      for (uint32_t t = sg.t0; t < sg.t1; ++t) bytes += sg.rec->terms[t].unpacked_length;
      base = std::min(base, sg.dst);
      top_addr = std::max<uintptr_t>(top_addr, sg.dst + bytes);
    }
    it.seg_chunk0.assign(ns + 1, 0);
    for (size_t sidx = 0; sidx < ns; ++sidx) {
      const Seg& sg = it.segs[sidx];
      it.at.sources[sidx].resize(sg.t1 - sg.t0);
      uint64_t off = 0, c = it.seg_chunk0[sidx];
      for (uint32_t i = sg.t0; i < sg.t1; ++i) {
        const auto& t = sg.rec->terms[i];
        const uint32_t n = uint32_t(t.range.end - t.range.start);
        it.gt.push_back({sidx, i, sg.dst - base + off, c, n, t.unpacked_length});
        off += t.unpacked_length;
        c += n;
      }
      it.seg_chunk0[sidx + 1] = c;
      it.at.chunk_lens[sidx].assign(size_t(c - it.seg_chunk0[sidx]), 0);
    }
    const size_t n = it.gt.size();
    const uint64_t nck = it.seg_chunk0[ns];
    it.dst = ns ? reinterpret_cast<uint8_t*>(base) : nullptr;
    it.dst_size = ns ? uint64_t(top_addr - base) : 0;
    it.hash_out = hashes + 32 * (ns ? it.segs[0].chunk0 : 0);
    it.size_out = sizes ? sizes + (ns ? it.segs[0].chunk0 : 0) : nullptr;
    // batches of whole terms that fit a slot (as in run_segments); a term larger than a slot grows
    // every slot, and the slots' record tables / device buffers grow to the largest batch -- both
    // only with the pipeline idle
    uint64_t max_bound = 0;
    for (size_t i = 0; i < n; ++i) max_bound = std::max(max_bound, term_bound(it.gt[i].ulen, it.gt[i].nchunks));
    if (max_bound > cap_) {
      s_drain();
      grow_staging(max_bound);
    }
    std::vector<SBatch> bs;
    bool first_of_pass;
    {
      std::lock_guard<std::mutex> g(smu_);
      first_of_pass = sbatch_total_ == sb0_;  // nothing submitted since the last reset
    }
    for (size_t next = 0; next < n;) {
      SBatch bt;
      bt.item = &it;
      bt.begin = next;
      uint64_t pos = 0;
      size_t end = next;
      const uint64_t cap_b = first_of_pass && bs.empty() ? first_batch_cap() : cap_;
      while (end < n) {
        const uint64_t bound = term_bound(it.gt[end].ulen, it.gt[end].nchunks);
        if (pos + bound > cap_b && end > next) break;
        bt.off.push_back(pos);
        pos += bound;
        ++end;
      }
      bt.end = end;
      bt.len.assign(end - next, 0);
      bt.src_at.assign(end - next, 0);
      bt.c_lo = it.gt[next].chunk;
      bt.c_hi = end < n ? it.gt[end].chunk : nck;
      bt.remaining = end - next;
      bs.push_back(std::move(bt));
      next = end;
    }
    size_t max_recs = 1, max_hs = 1;
    for (const SBatch& bt : bs) {
      uint64_t ub = 0;
      for (size_t i = bt.begin; i < bt.end; ++i) ub += it.gt[i].ulen;
      max_recs = std::max<size_t>(max_recs, size_t(bt.c_hi - bt.c_lo));
      max_hs = std::max(max_hs, zg_ingest_scratch_bytes(int(bt.c_hi - bt.c_lo), ub));
    }
    bool grow = false;
    for (const auto& sl : slots_) grow |= sl.rec_cap < max_recs || sl.chunks_dev.n < max_recs || sl.scratch.n < max_hs;
    if (grow) {
      s_drain();
      for (auto& sl : slots_) {
        if (sl.rec_cap < max_recs) {
          const size_t cap = std::max(max_recs, size_t(16384));
          if (!sl.rec_pin.alloc(cap * sizeof(ZgChunk))) throw Error("HipError", "pinning the chunk records failed");
          sl.rec_cap = cap;
        }
        sl.chunks_dev.ensure(std::max(max_recs, sl.rec_cap));
        sl.scratch.ensure(max_hs);
      }
    }
    hip_check(hipEventCreateWithFlags(&it.done, sync_event_flags()), "hipEventCreate");
    uint64_t ticket;
    {
      std::lock_guard<std::mutex> g(smu_);
      size_t unread = 0;
      for (auto& x : sitems_) unread += !x->collected;
      if (unread >= kErrRing) {
        (void)hipEventDestroy(it.done);
        throw Error("InvalidArgument", "too many pull items in flight");
      }
      ticket = ++sticket_;
      it.ticket = ticket;
      it.eslot = size_t(ticket % kErrRing);
      it.b0 = sbatch_total_;
      it.nb = bs.size();
      for (size_t k = 0; k < bs.size(); ++k) {
        for (size_t i = bs[k].begin; i < bs[k].end; ++i) swork_.emplace_back(sbatch_total_ + k, i);
        sbatches_.push_back(std::move(bs[k]));
      }
      sbatch_total_ += it.nb;
      if (it.nb == 0) it.queued = true;  // nothing to fetch (the caller still gets a done event)
      sitems_.push_back(std::move(item));
    }
    if (it.nb == 0) hip_check(hipEventRecord(it.done, stream_), "event");
    scv_.notify_all();
    return ticket;
  }

  void s_worker() {
    pthread_setname_np(pthread_self(), "zest-sfetch");  // (per-thread CPU time in /proc: bench.py)
    (void)hipSetDevice(device_);
    const size_t S = nslots_;
    while (true) {
      size_t g, i;
      SBatch* bp;
      {
        std::unique_lock<std::mutex> lk(smu_);
        scv_.wait(lk, [&] { return sstop_ || swork_next_ < swork_.size(); });
        if (sstop_) return;
        std::tie(g, i) = swork_[swork_next_++];
        bp = &sbatches_[g - sb0_];
        SItem& it = *bp->item;
        // Start-up: until the pass's first batch is queued, only its terms are fetched -- with every
        // worker free to run ahead, the first batch shared the host's copy bandwidth with 15 later
        // terms and the copy engine idled ~30 ms (4-rank rehearsal, profiles/r6/).  Afterwards the
        // workers run as far ahead as the free slots allow.  ZEST_STREAM_AHEAD = A > 0 keeps a
        // window of A batches past the oldest unqueued one for the whole pass; 0 turns both off.
        static const long ahead = [] {
          const char* v = std::getenv("ZEST_STREAM_AHEAD");
          return v && *v ? std::strtol(v, nullptr, 10) : -1L;
        }();
        scv_.wait(lk, [&] {
          if (sstop_ || it.failed) return true;
          if (sready_[g % S] < g) return false;
          if (ahead > 0) return g < ssubmit_next_ + size_t(ahead);
          return ahead == 0 || ssubmit_next_ > sb0_ || g == sb0_;
        });
        if (sstop_) return;
        if (it.failed) {  // the item is lost: its other terms need no fetch
          if (--bp->remaining == 0) scv_.notify_all();
          continue;
        }
        ++bp->copies;
      }
      SBatch& bt = *bp;
      SItem& it = *bt.item;
      Slot& s = slots_[g % S];
      const size_t j = i - bt.begin;
      try {
        const GTerm& gti = it.gt[i];
        const cas::Reconstruction& rec = *it.segs[gti.seg].rec;
        uint8_t* region = s.host + bt.off[j];
        const uint64_t room = (i + 1 < bt.end ? bt.off[j + 1] : cap_) - bt.off[j];
        FetchOptions topt;
        auto copied = [this, bp]() {
          {
            std::lock_guard<std::mutex> lk(smu_);
            --bp->copies;
          }
          scv_.notify_all();
        };
        if (sh_->writer) topt.on_copied = copied;
        ZgChunk* cr = s.recs() + (gti.chunk - bt.c_lo);
        uint32_t* lens = it.at.chunk_lens[gti.seg].data() + (gti.chunk - it.seg_chunk0[gti.seg]);
        const TermFetch tf = fetch_term_into(rec, gti, topt, copied, region, room, bt.off[j], uint32_t(j), cr, lens,
                                             it.at.sources[gti.seg][gti.term - it.segs[gti.seg].t0]);
        bt.src_at[j] = tf.src_at;
        bt.len[j] = tf.len;
        std::lock_guard<std::mutex> lk(smu_);
        if (!tf.planned) {
          it.at.planned_ok[gti.seg] = 0;
          if (!it.failed) {
            it.failed = true;
            it.err = "term range of " + it.jobs[gti.seg].xet_hash + " does not match its plan";
          }
        }
        if (--bt.remaining == 0) scv_.notify_all();
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(smu_);
        if (!it.failed) {
          it.failed = true;
          it.err = e.what();
        }
        if (--bt.remaining == 0) scv_.notify_all();
      }
    }
  }

  void s_submitter() {
    pthread_setname_np(pthread_self(), "zest-ssubmit");  // (per-thread CPU time in /proc: bench.py)
    (void)hipSetDevice(device_);
    const size_t S = nslots_;
    while (true) {
      size_t g;
      SBatch* bp;
      bool failed;
      {
        std::unique_lock<std::mutex> lk(smu_);
        scv_.wait(lk, [&] {
          if (sstop_) return true;
          if (ssubmit_next_ >= sb0_ + sbatches_.size() || ssubmit_next_ < sb0_) return false;
          const SBatch& b = sbatches_[ssubmit_next_ - sb0_];
          return b.remaining == 0 && sready_[ssubmit_next_ % S] >= ssubmit_next_;
        });
        if (sstop_) return;
        g = ssubmit_next_++;
        bp = &sbatches_[g - sb0_];
        failed = bp->item->failed;
      }
      SBatch& bt = *bp;
      SItem& it = *bt.item;
      const size_t slot = g % S;
      Slot& s = slots_[slot];
      const bool first = g == it.b0, last = g + 1 == it.b0 + it.nb;
      std::string err;
      try {
        trace::Span sp("device", "stream: queue H2D + place/hash");
        if (first) hip_check(hipMemsetAsync(serr_.p + it.eslot, 0, sizeof(unsigned long long), stream_), "hipMemset");
        if (!failed) {
          uint64_t top = 0, fetched = 0;
          for (size_t j = 0; j < bt.len.size(); ++j) {
            top = std::max<uint64_t>(top, bt.src_at[j] + bt.len[j]);
            fetched += bt.len[j];
            it.at.seg_fetched[it.gt[bt.begin + j].seg] += bt.len[j];
          }
          it.at.fetched += fetched;
          const int nchunks = int(bt.c_hi - bt.c_lo);
          uint64_t ubytes = 0;
          for (size_t i = bt.begin; i < bt.end; ++i) ubytes += it.gt[i].ulen;
          bool compressed = false;
          for (int c = 0; c < nchunks && !compressed; ++c) compressed = s.recs()[c].scheme != 0;
          const size_t hs_bytes = zg_ingest_scratch_bytes(nchunks, ubytes);
          if (skern_set_[slot]) hip_check(hipStreamWaitEvent(copy_stream_, skern_[slot], 0), "hipStreamWaitEvent");
          if (timing_)
            for (auto& e : bt.tev) hip_check(hipEventCreate(&e), "hipEventCreate");
          if (timing_) hip_check(hipEventRecord(bt.tev[0], copy_stream_), "event");
          static const uint64_t merge_gap = env_size("ZEST_H2D_MERGE_GAP", size_t(64) << 10);
          for (const auto& [lo, hi] : copy_ranges(bt.src_at, bt.len, merge_gap)) {
            hip_check(hipMemcpyAsync(s.dev.p + lo, s.host + lo, hi - lo, hipMemcpyHostToDevice, copy_stream_), "H2D");
            bt.h2d += hi - lo;
          }
          if (nchunks)
            hip_check(hipMemcpyAsync(s.chunks_dev.p, s.recs(), sizeof(ZgChunk) * size_t(nchunks), hipMemcpyHostToDevice,
                                     copy_stream_),
                      "H2D chunk records");
          hip_check(hipEventRecord(sh2d_[slot], copy_stream_), "event");
          if (timing_) hip_check(hipEventRecord(bt.tev[1], copy_stream_), "event");
          hip_check(hipStreamWaitEvent(stream_, sh2d_[slot], 0), "hipStreamWaitEvent");
          if (timing_) hip_check(hipEventRecord(bt.tev[2], stream_), "event");
          hip_check(zg_ingest_chunks(s.dev.p, top, it.dst, it.dst_size, s.chunks_dev.p, nchunks, compressed ? 1 : 0,
                                     serr_.p + it.eslot, it.hash_out + 32 * bt.c_lo,
                                     it.size_out ? it.size_out + bt.c_lo : nullptr, 0, s.scratch.p, hs_bytes, stream_),
                    "ingest");
          if (timing_) hip_check(hipEventRecord(bt.tev[3], stream_), "event");
          hip_check(hipEventRecord(skern_[slot], stream_), "event");
          skern_set_[slot] = 1;
          bt.gpu = true;
        }
      } catch (const std::exception& e) {
        err = e.what();
      }
      if (last) {
        (void)hipMemcpyAsync(reinterpret_cast<unsigned long long*>(serr_host_.data()) + it.eslot, serr_.p + it.eslot,
                             sizeof(unsigned long long), hipMemcpyDeviceToHost, stream_);
        if (hipEventRecord(it.done, stream_) != hipSuccess && err.empty()) err = "hipEventRecord (item done)";
      }
      {
        std::lock_guard<std::mutex> lk(smu_);
        if (!err.empty() && !it.failed) {
          it.failed = true;
          it.err = err;
        }
        sissued_.push_back(g);
        if (last) it.queued = true;
      }
      scv_.notify_all();
    }
  }

  void s_releaser() {
    pthread_setname_np(pthread_self(), "zest-srelease");  // (per-thread CPU time in /proc: bench.py)
    (void)hipSetDevice(device_);
    const size_t S = nslots_;
    while (true) {
      size_t g;
      SBatch* bp;
      {
        std::unique_lock<std::mutex> lk(smu_);
        scv_.wait(lk, [&] { return sstop_ || !sissued_.empty(); });
        if (sissued_.empty()) return;  // stopping
        g = sissued_.front();
        sissued_.pop_front();
        bp = &sbatches_[g - sb0_];
      }
      const bool ok = !bp->gpu || gpu::idle_event_sync(sh2d_[g % S]) == hipSuccess;
      {
        std::unique_lock<std::mutex> lk(smu_);
        if (!ok && !bp->item->failed) {
          bp->item->failed = true;
          bp->item->err = "hipEventSynchronize (H2D)";
        }
        // the write-behind writer's copy threads are done with the slot
        scv_.wait(lk, [&] { return sstop_ || bp->copies == 0; });
        sready_[g % S] = g + S;
        ++sreleased_;
      }
      scv_.notify_all();
    }
  }

  struct ItemResult {
    std::string err;                      // empty: every term fetched and matched its plan
    std::vector<TermJobResult> results;   // per job
    uintptr_t event = 0;                  // hipEvent_t: the item's kernels (and error word copy) done
  };

  // Blocks until the item's last batch is queued on the GPU (or the item failed).  Settles the
  // bookkeeping like pull_terms: runs go to the settle book, or a failed item's quarantined peer
  // runs (and the runs of ranges that did not match their plan) are dropped.
  ItemResult wait_item(uint64_t ticket) {
    SItem* itp;
    {
      std::unique_lock<std::mutex> lk(smu_);
      itp = s_find(ticket);
      scv_.wait(lk, [&] { return itp->queued; });
      if (itp->collected) throw Error("InvalidArgument", "pull ticket " + std::to_string(ticket) + " already waited");
      itp->collected = true;
    }
    SItem& it = *itp;
    ItemResult out;
    out.event = reinterpret_cast<uintptr_t>(it.done);
    out.results.resize(it.segs.size());
    if (it.failed) {
      out.err = it.err.empty() ? "fetch failed" : it.err;
      for (size_t k = 0; k < it.segs.size(); ++k)
        for (size_t t = 0; t < it.at.sources[k].size(); ++t) {
          const TermSource& ts = it.at.sources[k][t];
          if (!it.at.planned_ok[k])
            sh_->bridge->settle(it.segs[k].rec->terms[it.segs[k].t0 + t].hash_hex, ts.src, ts.run_offset, ts.pending,
                                false);
          else if (ts.src == Source::Peer && !ts.pending.empty())
            sh_->bridge->settle(std::string(), ts.src, ts.run_offset, ts.pending, false);
        }
      return out;
    }
    for (size_t k = 0; k < it.segs.size(); ++k) {
      TermJobResult& r = out.results[k];
      r.chunk_lens = std::move(it.at.chunk_lens[k]);
      r.fetched = it.at.seg_fetched[k];
      for (size_t t = 0; t < it.at.sources[k].size(); ++t) {
        const TermSource& ts = it.at.sources[k][t];
        const cas::Term& term = it.segs[k].rec->terms[it.segs[k].t0 + t];
        sh_->book.add(it.jobs[k].xet_hash, term.hash_hex, ts.src, ts.run_offset, ts.pending);
        (ts.src == Source::Peer ? r.from_peer : ts.src == Source::Cache ? r.from_cache : r.from_cdn) +=
            term.unpacked_length;
      }
    }
    return out;
  }

  // The item's device error word (0: every chunk decoded and placed); waits for its kernels.
  unsigned long long item_error(uint64_t ticket) {
    SItem* itp;
    {
      std::lock_guard<std::mutex> lk(smu_);
      itp = s_find(ticket);
      if (!itp->queued) throw Error("InvalidArgument", "item_error before wait_item");
    }
    hip_check(gpu::idle_event_sync(itp->done), "hipEventSynchronize (item)");
    return reinterpret_cast<volatile unsigned long long*>(serr_host_.data())[itp->eslot];
  }

  // Device timeline of the last timed pass: intervals [copy start, copy end] and [kernels start,
  // kernels end] per batch (ms from the first copy), their unions, and the time both ran at once.
  void record_timeline(hipEvent_t* tev, size_t nb, uint64_t h2d_bytes) {
    std::vector<std::array<hipEvent_t, 4>> ev(nb);
    for (size_t b = 0; b < nb; ++b) ev[b] = {tev[4 * b], tev[4 * b + 1], tev[4 * b + 2], tev[4 * b + 3]};
    record_timeline(ev, h2d_bytes);
  }
  // (copy start, copy end, kernels start, kernels end) per batch, relative to the first copy start
  void record_timeline(const std::vector<std::array<hipEvent_t, 4>>& tev, uint64_t h2d_bytes) {
    const size_t nb = tev.size();
    if (!nb) return;
    std::vector<std::pair<double, double>> cp, kn;
    for (size_t b = 0; b < nb; ++b) {
      float a = 0, c = 0, d = 0, e = 0;
      if (hipEventElapsedTime(&a, tev[0][0], tev[b][0]) != hipSuccess ||
          hipEventElapsedTime(&c, tev[0][0], tev[b][1]) != hipSuccess ||
          hipEventElapsedTime(&d, tev[0][0], tev[b][2]) != hipSuccess ||
          hipEventElapsedTime(&e, tev[0][0], tev[b][3]) != hipSuccess)
        return;
      cp.emplace_back(a, c);
      kn.emplace_back(d, e);
    }
    auto unite = [](std::vector<std::pair<double, double>> v) {
      std::sort(v.begin(), v.end());
      std::vector<std::pair<double, double>> u;
      for (auto& x : v)
        if (!u.empty() && x.first <= u.back().second) u.back().second = std::max(u.back().second, x.second);
        else u.push_back(x);
      return u;
    };
    auto total = [](const std::vector<std::pair<double, double>>& u) {
      double t = 0;
      for (auto& x : u) t += x.second - x.first;
      return t;
    };
    const auto uc = unite(cp), uk = unite(kn);
    double both = 0;
    for (size_t i = 0, j = 0; i < uc.size() && j < uk.size();) {
      const double lo = std::max(uc[i].first, uk[j].first), hi = std::min(uc[i].second, uk[j].second);
      if (hi > lo) both += hi - lo;
      (uc[i].second < uk[j].second) ? ++i : ++j;
    }
    const double window = std::max(uc.back().second, uk.back().second);
    std::lock_guard<std::mutex> g(timeline_mu_);
    timeline_ = "{\"batches\":" + std::to_string(nb) + ",\"window_ms\":" + std::to_string(window) +
                ",\"h2d_busy_ms\":" + std::to_string(total(uc)) + ",\"kernel_busy_ms\":" + std::to_string(total(uk)) +
                ",\"overlap_ms\":" + std::to_string(both) + ",\"h2d_bytes\":" + std::to_string(h2d_bytes) +
                ",\"h2d_GBps_busy\":" + std::to_string(total(uc) > 0 ? double(h2d_bytes) / total(uc) / 1e6 : 0.0) + "}";
  }

  hipEvent_t* take_timing_events(size_t n) {
    while (timing_events_.size() < n) {
      hipEvent_t e = nullptr;
      hip_check(hipEventCreate(&e), "hipEventCreate");
      timing_events_.push_back(e);
    }
    return timing_events_.data();
  }

  std::string timeline_json() {
    std::lock_guard<std::mutex> g(timeline_mu_);
    return timeline_.empty() ? "{}" : timeline_;
  }

  uint64_t first_batch_cap() const {
    static const uint64_t mb = env_size("ZEST_FIRST_BATCH_MB", 128);
    return mb ? std::min<uint64_t>(cap_, mb << 20) : cap_;
  }

  // Upper bound of a term's fetched bytes: Xet stores a chunk uncompressed when compression does
  // not help, so the payload is <= its unpacked size plus LZ4 frame overhead; + 8-byte headers.
  static uint64_t term_bound(uint64_t unpacked, uint64_t nchunks) {
    return unpacked + unpacked / 128 + 80 * nchunks + 4096;
  }

  void grow_staging(uint64_t bytes) {
    hip_check(hipStreamSynchronize(copy_stream_), "sync");  // no copy still reads the old buffers
    hip_check(hipStreamSynchronize(stream_), "sync");
    for (auto& s : slots_) {
      s.host = nullptr;
      if (!s.pin.alloc(bytes + 4096)) throw Error("HipError", "pinning the staging buffer failed");
      s.host = s.pin.data();
      s.dev.ensure(bytes);
    }
    cap_ = bytes;
  }

  std::shared_ptr<Shared> sh_;
  int device_;
  size_t cap_;
  int threads_;
  size_t nslots_;
  hipStream_t stream_ = nullptr;       // kernels
  hipStream_t copy_stream_ = nullptr;  // H2D copies
  std::mutex init_mu_;
  bool device_ready_ = false;
  std::vector<Slot> slots_;
  std::vector<hipEvent_t> events_;
  const bool timing_ = [] {
    const char* v = std::getenv("ZEST_DEVICE_TIMING");
    return v && std::string(v) == "1";
  }();
  std::vector<hipEvent_t> timing_events_;
  std::mutex timeline_mu_;
  std::string timeline_;
  DevBuf<unsigned long long> err_;
  // streaming engine (submit_terms)
  bool s_started_ = false;
  std::mutex smu_;
  std::condition_variable scv_;
  bool sstop_ = false;
  std::deque<std::unique_ptr<SItem>> sitems_;
  std::deque<SBatch> sbatches_;                   // global batch g at sbatches_[g - sb0_]
  size_t sb0_ = 0, sbatch_total_ = 0, sreleased_ = 0, ssubmit_next_ = 0;
  std::deque<std::pair<size_t, size_t>> swork_;  // (global batch, item term) in fetch order
  size_t swork_next_ = 0;
  std::deque<size_t> sissued_;                   // batches queued on the GPU, for the releaser
  std::vector<size_t> sready_;                   // per slot: first batch allowed to fill it
  std::vector<hipEvent_t> sh2d_, skern_;         // per slot: last batch's H2D landed / kernels ran
  std::vector<uint8_t> skern_set_;
  std::vector<std::thread> sworkers_;
  std::thread ssubmitter_, sreleaser_;
  DevBuf<unsigned long long> serr_;
  PinnedBuf serr_host_;
  uint64_t sticket_ = 0;
  DevBuf<uint8_t> hashes_;
  DevBuf<uint64_t> sizes_;
  DevBuf<ZgMerkleJob> merkle_job_;
  DevBuf<uint8_t> merkle_scratch_;
  DevBuf<uint8_t> root_;
};


DeviceXetPull::DeviceXetPull(const DevicePullOptions& opt) : impl_(std::make_unique<Impl>(opt, nullptr)) {}
DeviceXetPull::DeviceXetPull(const DevicePullOptions& opt, std::shared_ptr<Shared> shared)
    : impl_(std::make_unique<Impl>(opt, std::move(shared))) {}
std::unique_ptr<DeviceXetPull> DeviceXetPull::sibling(size_t staging_bytes, int slots) const {
  DevicePullOptions o;
  o.device = impl_->device_;
  o.staging_bytes = staging_bytes ? staging_bytes : impl_->cap_;
  o.threads = impl_->threads_;
  o.slots = slots;
  o.defer_device = true;
  return std::unique_ptr<DeviceXetPull>(new DeviceXetPull(o, impl_->sh_));
}
DeviceXetPull::~DeviceXetPull() = default;

std::vector<PullFileStats> DeviceXetPull::pull_files(const std::vector<PullRequest>& files,
                                                     const PullProgressFn& progress) {
  std::vector<std::tuple<std::string, uintptr_t, uint64_t>> f;
  f.reserve(files.size());
  for (const auto& r : files) f.emplace_back(r.xet_hash, r.dst, r.size);
  impl_->progress_ = progress;
  struct Reset {
    PullProgressFn& p;
    ~Reset() { p = nullptr; }
  } reset{impl_->progress_};
  return impl_->pull_files(f);
}

std::vector<TermJobResult> DeviceXetPull::pull_terms(const std::vector<TermJob>& jobs, uint8_t* hashes, uint64_t* sizes,
                                                     bool repair) {
  return impl_->pull_terms(jobs, hashes, sizes, repair);
}
uint64_t DeviceXetPull::submit_terms(const std::vector<TermJob>& jobs, uint8_t* hashes, uint64_t* sizes) {
  return impl_->submit_terms(jobs, hashes, sizes);
}
DeviceXetPull::ItemResult DeviceXetPull::wait_item(uint64_t ticket) {
  auto r = impl_->wait_item(ticket);
  return ItemResult{std::move(r.err), std::move(r.results), r.event};
}
unsigned long long DeviceXetPull::item_error(uint64_t ticket) { return impl_->item_error(ticket); }
void DeviceXetPull::stream_reset(bool cancel) { impl_->s_reset(cancel); }
void DeviceXetPull::order_after(uintptr_t event) { impl_->order_after(reinterpret_cast<hipEvent_t>(event)); }
size_t DeviceXetPull::settle(const std::string& xet_hash, bool ok) { return impl_->settle(xet_hash, ok); }
std::vector<TermShape> DeviceXetPull::term_shapes(const std::string& xet_hash) { return impl_->term_shapes(xet_hash); }
std::vector<TermKey> DeviceXetPull::term_keys(const std::string& xet_hash) { return impl_->sh_->recs->keys(xet_hash); }
std::vector<uint8_t> DeviceXetPull::cached_terms(const std::vector<std::string>& hexes,
                                                 const std::vector<uint32_t>& starts, const std::vector<uint32_t>& ends) {
  return zest::cached_terms(*impl_->sh_->cache, hexes, starts, ends, impl_->threads_);
}
void DeviceXetPull::reset_reconstructions() { impl_->sh_->recs->clear(); }
void DeviceXetPull::init_device() { impl_->init_device(); }
void DeviceXetPull::flush_cache_writes() { impl_->flush_cache_writes(); }
std::string DeviceXetPull::timeline_json() const { return impl_->timeline_json(); }
std::string DeviceXetPull::cache_writer_json() const {
  auto* w = impl_->sh_->writer.get();
  if (!w) return "{}";
  const auto st = w->stats();
  return "{\"queued_bytes\":" + std::to_string(st.queued_bytes) + ",\"written_bytes\":" + std::to_string(st.written_bytes) +
         ",\"dropped_bytes\":" + std::to_string(st.dropped_bytes) +
         ",\"deferred_runs\":" + std::to_string(impl_->sh_->bridge->deferred_count()) + "}";
}
std::string DeviceXetPull::stats_json() const { return impl_->stats_json(); }
size_t DeviceXetPull::staging_bytes() const { return impl_->staging_bytes(); }

}  // namespace zest::gpurt
