#include "pull.h"

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <thread>

#include <fcntl.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <iomanip>
#include <optional>

#include "bridge.h"
#include "downloader.h"
#include "http.h"
#include "json.h"
#include "trace.h"
#include "hub.h"
#include "storage.h"
#include "swarm.h"

extern char** environ;

namespace zest {

void PullProgress::add(size_t file, uint64_t n, int source) {
  if (file < files.size()) {  // a repair refetch re-adds terms: clamp each file at its size
    File& f = *files[file];
    uint64_t cur = f.done.load();
    uint64_t next;
    do {
      next = std::min<uint64_t>(f.size ? f.size : cur + n, cur + n);
    } while (!f.done.compare_exchange_weak(cur, next));
    bytes += next - cur;
  } else {
    bytes += n;
  }
  (source == 1 ? from_cache : source == 2 ? from_peer : from_cdn) += n;
  last_source = source;
}

const char* PullProgress::source_name(int s) {
  return s == 1 ? "cache" : s == 2 ? "peer" : s == 3 ? "cdn" : "none";
}

namespace {
int source_code(Source s) { return s == Source::Cache || s == Source::Resumed ? 1 : s == Source::Peer ? 2 : 3; }
}  // namespace

bool server_healthy(uint16_t http_port, int timeout_ms) {
  try {
    http::RequestOptions o;
    o.timeout_ms = timeout_ms;
    o.max_redirects = 0;
    auto r = http::get("http://127.0.0.1:" + std::to_string(http_port) + "/v1/health", {}, o);
    return r.status == 200;
  } catch (const Error&) {
    return false;
  }
}

bool spawn_background_server(const std::string& self_exe, uint16_t http_port) {
  if (server_healthy(http_port, 300)) return true;
  std::string port = std::to_string(http_port);
  const char* argv[] = {self_exe.c_str(), "serve", "--http-port", port.c_str(), nullptr};
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  posix_spawn_file_actions_addopen(&fa, 1, "/dev/null", O_WRONLY, 0);
  posix_spawn_file_actions_addopen(&fa, 2, "/dev/null", O_WRONLY, 0);
  posix_spawnattr_t at;
  posix_spawnattr_init(&at);
  posix_spawnattr_setflags(&at, POSIX_SPAWN_SETSID);
  pid_t pid = 0;
  int rc = posix_spawn(&pid, self_exe.c_str(), &fa, &at, const_cast<char* const*>(argv), environ);
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&at);
  return rc == 0;
}

PullSummary run_pull(Config& cfg, const PullOptions& opt, std::ostream& out, std::ostream& err) {
  const auto t0 = std::chrono::steady_clock::now();
  PullSummary S;
  out << "zest pull " << opt.repo_id << " (revision: " << opt.revision << ")\n";
  if (!cfg.hf_token) err << "Warning: no HuggingFace token found. Set HF_TOKEN or run `huggingface-cli login`.\n";
  if (opt.p2p) out << "P2P enabled (peer_id: " << peer_id::kClientPrefix << "...)\n";
  else out << "P2P disabled (CDN only)\n";
  out << "Fetching model info from HuggingFace Hub...\n" << std::flush;
  std::optional<trace::Span> listing_span(std::in_place, "pull", "list files + resolve commit");
  std::vector<hub::RepoFile> files = hub::list_files(cfg, opt.repo_id, opt.revision, opt.repo_type);
  if (!opt.include.empty()) {
    std::vector<hub::RepoFile> keep;
    for (auto& f : files)
      for (auto& suf : opt.include)
        if (f.path.size() >= suf.size() && f.path.compare(f.path.size() - suf.size(), suf.size(), suf) == 0) {
          keep.push_back(f);
          break;
        }
    files.swap(keep);
  }
  auto sha = hub::resolve_commit(cfg, opt.repo_id, opt.revision, opt.repo_type);
  S.commit = sha ? *sha : opt.revision;
  listing_span.reset();
  if (sha) out << "Found " << files.size() << " files (revision: " << opt.revision << " \xE2\x86\x92 " << S.commit << ")\n";
  else out << "Found " << files.size() << " files (revision: " << opt.revision << ")\n";
  out << "Detecting Xet-backed files...\n";
  for (auto& f : files)
    if (f.xet_hash) S.xet_files++;
  out << "  " << S.xet_files << " Xet-backed files, " << files.size() << " total files\n";
  S.files = files.size();
  PullProgress* prog = opt.progress.get();
  if (prog) {
    std::lock_guard<std::mutex> g(prog->mu);
    for (auto& f : files) {
      auto pf = std::make_unique<PullProgress::File>();
      pf->path = f.path;
      pf->size = f.size;
      prog->total += f.size;
      prog->files.push_back(std::move(pf));
    }
    prog->listed = true;
  }
  auto set_state = [&](size_t i, int st) {
    if (prog && i < prog->files.size()) prog->files[i]->state = st;
  };

  std::vector<net::Addr> boot;
  for (auto& b : opt.dht_bootstrap) {
    try {
      boot.push_back(net::Addr::parse(b, 6881));
    } catch (const Error&) {
      err << "Warning: invalid DHT bootstrap node: " << b << "\n";
    }
  }
  std::optional<trace::Span> setup_span(std::in_place, "pull", "cache scan + swarm + auth");
  storage::XorbRegistry registry;
  registry.scan(cfg);
  storage::XorbCache cache(cfg, &registry);
  cache.set_registry_lookup(true);  // misses answered from the scan + this pull's own puts (no directory listing per term)
  SwarmDownloader swarm(cfg, opt.tracker, opt.p2p, opt.dht && opt.p2p, boot);
  for (auto& p : opt.peers) {
    try {
      swarm.add_direct_peer(net::Addr::parse(p, 6881));
      out << "  Direct peer: " << p << "\n";
    } catch (const Error&) {
      err << "Warning: invalid peer address: " << p << "\n";
    }
  }
  XetBridge bridge(cfg, &cache, &swarm);
  if (S.xet_files > 0) {
    out << "Authenticating with Xet CAS...\n" << std::flush;
    try {
      bridge.authenticate(opt.repo_id, opt.repo_type, opt.revision);
    } catch (const Error& e) {
      err << "Warning: Xet auth failed (" << e.what() << ")\n";
    }
  }
  ParallelDownloader dl(bridge, opt.concurrency > 0 ? opt.concurrency : int(cfg.concurrency));
  setup_span.reset();
  S.snapshot_dir = cfg.snapshot_dir(opt.repo_id, S.commit);
  size_t k = 0;
  std::vector<uint8_t> ok(files.size(), 1);
  struct XetJob {
    size_t file;
    std::string dst;
  };
  std::vector<XetJob> xet_jobs;
  for (auto& f : files) {
    ++k;
    uint8_t& file_ok = ok[k - 1];
    out << "[" << k << "/" << files.size() << "] " << f.path;
    const std::string dst = S.snapshot_dir + "/" + f.path;
    if (storage::exists(dst) && (f.size == 0 || storage::file_size(dst) == f.size)) {
      // Xet files must also match their verified marker (or re-hash to the published hash):
      // size alone would keep a corrupted or truncated-then-extended copy forever.
      bool good = true;
      if (f.xet_hash && opt.verify &&
          !storage::check_verified_marker(cfg, opt.repo_id, S.commit, f.path, *f.xet_hash, dst)) {
        try {
          good = storage::xet_hash_of_file(dst) == *f.xet_hash;
        } catch (const Error&) {
          good = false;
        }
        if (good) storage::write_verified_marker(cfg, opt.repo_id, S.commit, f.path, *f.xet_hash, dst);
      }
      if (good) {
        out << " (cached)\n";
        S.cached_files++;
        set_state(k - 1, 4);
        if (prog) prog->add(k - 1, f.size, 1);
        continue;
      }
      out << " (cached copy failed verification, downloading again)";
      storage::remove_file(dst);
    }
    if (f.xet_hash) {
      out << " [xet]\n" << std::flush;
      if (!bridge.authenticated()) {
        err << "  Error downloading via xet: not authenticated\n";
        file_ok = 0;
        continue;
      }
      xet_jobs.push_back({k - 1, dst});
    } else {
      out << " [regular]\n" << std::flush;
      set_state(k - 1, 1);
      try {
        const uint64_t n = hub::download_regular(cfg, opt.repo_id, S.commit == opt.revision ? opt.revision : S.commit, f.path, dst);
        S.bytes += n;
        if (prog) prog->add(k - 1, n, 3);
        set_state(k - 1, 2);
      } catch (const Error& e) {
        err << "  Error downloading: " << e.what() << "\n";
        file_ok = 0;
        set_state(k - 1, 3);
        continue;
      }
    }
  }
  // Xet files: up to ZEST_FILE_CONCURRENCY (default 4) at once.  Their terms share the
  // downloader's `concurrency` slots, so a file's tail overlaps the next file's terms, and the
  // snapshot writes spread over several files (concurrent pwrites to ONE file serialize on its
  // inode: Llama-3.1-8B from one HBM peer spent 13 s of 34 thread-seconds in pwrite at 3.75 GB/s,
  // profiles/host_pull_trace_r2.md).
  {
    const char* fc = std::getenv("ZEST_FILE_CONCURRENCY");
    const size_t nfile_threads = std::max<size_t>(1, std::min<size_t>(fc ? std::strtoul(fc, nullptr, 10) : 4,
                                                                       xet_jobs.size()));
    std::atomic<size_t> next{0};
    std::atomic<uint64_t> bytes{0};
    std::mutex io_mu;
    auto run = [&]() {
      for (size_t j; (j = next.fetch_add(1)) < xet_jobs.size();) {
        const XetJob& job = xet_jobs[j];
        const hub::RepoFile& f = files[job.file];
        try {
          trace::Span fs("pull", "xet file");
          set_state(job.file, 1);
          std::function<void(uint64_t, Source)> on_term;
          if (prog)
            on_term = [prog, &job, &swarm](uint64_t n, Source src) {
              prog->add(job.file, n, source_code(src));
              prog->peers = uint32_t(swarm.stats().peers_connected.load());
            };
          FileResult r = dl.reconstruct_to_file(*f.xet_hash, job.dst, opt.verify, on_term);
          set_state(job.file, 2);
          bytes += r.bytes;
          if (r.verified) storage::write_verified_marker(cfg, opt.repo_id, S.commit, f.path, *f.xet_hash, job.dst);
          if (r.resumed_terms) {
            std::lock_guard<std::mutex> g(io_mu);
            out << "  " << f.path << ": resumed " << r.resumed_terms << "/" << r.terms << " terms\n";
          }
        } catch (const Error& e) {
          std::lock_guard<std::mutex> g(io_mu);
          err << "  Parallel download error (" << f.path << ": " << e.what() << ")\n";
          ok[job.file] = 0;
          set_state(job.file, 3);
        }
      }
    };
    std::vector<std::thread> fts;
    for (size_t t = 1; t < nfile_threads; ++t) fts.emplace_back(run);
    run();
    for (auto& t : fts) t.join();
    S.bytes += bytes.load();
  }
  if (cfg.cache_max_gb > 0) {  // size-bounded xorb cache: drop least recently used runs
    const uint64_t cut = cache.trim(uint64_t(cfg.cache_max_gb * 1e9));
    if (cut) out << "Trimmed the xorb cache by " << std::fixed << std::setprecision(1) << double(cut) / 1e6
                 << " MB (ZEST_CACHE_MAX_GB=" << cfg.cache_max_gb << ")\n";
  } else {
    cache.sweep_pending();  // quarantine runs orphaned by pulls that died
  }
  try {
    storage::write_ref(cfg, opt.repo_id, opt.revision, S.commit);
  } catch (const Error& e) {
    err << "Warning: failed to write ref: " << e.what() << "\n";
  }
  bridge.print_stats(out);
  swarm.print_stats(out);
  S.bytes_from_peer = bridge.stats().bytes_from_peer;
  S.bytes_from_cdn = bridge.stats().bytes_from_cdn;
  S.bytes_from_cache = bridge.stats().bytes_from_cache;
  S.stats_json = bridge.stats_json();
  json::Writer fw;
  fw.arr();
  for (size_t i = 0; i < files.size(); ++i) {
    fw.obj().key("path").str(files[i].path).key("size").num_u(files[i].size).key("xet_hash");
    if (files[i].xet_hash) fw.str(*files[i].xet_hash);
    else fw.null();
    fw.key("ok").boolean(ok[i] != 0).end();
    if (!ok[i]) S.failed_files++;
  }
  fw.end();
  S.files_json = fw.out();
  S.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  out << "\nDone! Model available at:\n  " << S.snapshot_dir << "\n";
  out << "\nRun: transformers.AutoModel.from_pretrained(\"" << opt.repo_id << "\")\n" << std::flush;
  return S;
}

}  // namespace zest
