// `zest-gpu-worker`: one process per GPU for `zest pull <repo> --gpus N` (started by the CLI with
// HIP_VISIBLE_DEVICES pinned to one device).  Native end to end -- no Python or torch start-up on
// the path, no torchrun agent and no RCCL communicator (files are independent, so the workers never
// talk to each other; the CLI aggregates their status files).
//
//   list files (Hub API) -> this worker's Xet files (LPT by size over ZEST_GPU_WORLD workers)
//   -> skip verified cached files -> device-direct pull of all of them in one call (DeviceXetPull:
//   fetch -> pinned -> H2D -> GPU decode + BLAKE3 + Merkle verify into HBM) -> snapshot write-back
//   streaming behind the pull (64 MiB pieces, D2H + pwrite threads, into `.incomplete` files that
//   are renamed once the pull verified them).
//
// Environment: ZEST_GPU_RANK / ZEST_GPU_WORLD (this worker's index and the worker count),
// ZEST_GPU_STATUS (path of this worker's JSON status: written only when the worker ran to the end).
// Reference: the host pull it replaces for GPU nodes is main.zig:83-305 (cmdPull).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <iostream>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "config.h"
#include "device_pull.h"
#include "hub.h"
#include "json.h"
#include "pinned.h"
#include "storage.h"
#include "trace.h"

using namespace zest;

namespace {

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error("HipError", std::string(what) + ": " + hipGetErrorString(e));
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int env_int(const char* k, int def) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : def;
}

// LPT greedy, identical on every worker: largest file to the least-loaded worker (ties: lower index).
std::vector<int> assign_owners(const std::vector<uint64_t>& sizes, int world) {
  std::vector<size_t> order(sizes.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return sizes[a] > sizes[b]; });
  std::vector<uint64_t> load(size_t(std::max(1, world)), 0);
  std::vector<int> owner(sizes.size(), 0);
  for (size_t i : order) {
    const size_t r = size_t(std::min_element(load.begin(), load.end()) - load.begin());
    owner[i] = int(r);
    load[r] += sizes[i];
  }
  return owner;
}

// Snapshot write-back that streams while the device pull runs: the pull reports, after each
// staging batch, how much of each file is in HBM (PullProgressFn); those bytes are queued as pieces,
// and `threads` writers each copy a piece to a pinned buffer (own stream) and pwrite it into the
// file's `.incomplete` temp file.  The file is renamed into the snapshot only once the whole pull
// call verified it.  A buffered pwrite holds the file's inode lock, so one file takes ~10 GB/s on
// the box (profiles/write_probe_box_r3.jsonl) -- below the ~14 GB/s the pull delivers -- but the
// files of a pull arrive one after the other and their writes overlap each other.
class WriteBack {
 public:
  struct File {
    std::string dst, tmp;
    const uint8_t* dev = nullptr;
    uint64_t size = 0, queued = 0;
    int fd = -1;
    bool repaired = false;  // a repair pass overwrote its bytes: written again after the pull
    size_t pending = 0;     // pieces queued or being written
    std::string err;
  };

  WriteBack(int threads, size_t piece) : piece_(piece) {
    for (int t = 0; t < threads; ++t) {
      Lane l;
      hip_ok(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking), "hipStreamCreate");
      l.pin = std::make_shared<gpurt::PinnedBuf>();
      if (!l.pin->alloc(piece_)) throw Error("HipError", "pinning a write-back buffer failed");
      l.host = l.pin->data();
      lanes_.push_back(l);
    }
  }
  ~WriteBack() { stop(); }  // pinned buffers and streams go with the process (the worker _Exits)

  void start(std::vector<File>* files) {
    files_ = files;
    closing_ = false;
    for (size_t t = 0; t < lanes_.size(); ++t) threads_.emplace_back([this, t] { loop(lanes_[t]); });
  }
  // PullProgressFn: file f holds [0, bytes) in HBM after a batch of attempt `attempt`
  void progress(size_t f, int attempt, uint64_t bytes) {
    std::lock_guard<std::mutex> g(mu_);
    File& fl = (*files_)[f];
    if (attempt > 0) {
      fl.repaired = true;
      return;
    }
    post_locked(f, fl.queued, bytes);
    fl.queued = std::max(fl.queued, bytes);
  }
  void post(size_t f, uint64_t lo, uint64_t hi) {
    std::lock_guard<std::mutex> g(mu_);
    post_locked(f, lo, hi);
  }
  void drain() {
    std::unique_lock<std::mutex> g(mu_);
    idle_.wait(g, [&] { return pending_ == 0; });
  }
  // Wait until every piece queued for files `ks` is on its way to the disk (pwritten).
  void wait_files(const std::vector<size_t>& ks) {
    std::unique_lock<std::mutex> g(mu_);
    idle_.wait(g, [&] {
      for (size_t k : ks)
        if ((*files_)[k].pending) return false;
      return true;
    });
  }
  bool repaired(size_t k) {
    std::lock_guard<std::mutex> g(mu_);
    return (*files_)[k].repaired;
  }
  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      closing_ = true;
      work_.notify_all();
    }
    for (auto& t : threads_) t.join();
    threads_.clear();
  }

 private:
  struct Lane {
    hipStream_t stream = nullptr;
    std::shared_ptr<gpurt::PinnedBuf> pin;
    uint8_t* host = nullptr;
  };
  struct Piece {
    size_t file;
    uint64_t off, len;
  };
  void post_locked(size_t f, uint64_t lo, uint64_t hi) {
    for (uint64_t o = lo; o < hi; o += piece_) {
      q_.push_back({f, o, std::min<uint64_t>(piece_, hi - o)});
      ++pending_;
      ++(*files_)[f].pending;
    }
    work_.notify_all();
  }
  void loop(Lane& l) {
    while (true) {
      Piece p;
      {
        std::unique_lock<std::mutex> g(mu_);
        work_.wait(g, [&] { return closing_ || !q_.empty(); });
        if (q_.empty()) return;
        p = q_.front();
        q_.pop_front();
      }
      File& fl = (*files_)[p.file];
      std::string e;
      {
        trace::Span sp("write", "D2H piece");
        if (hipMemcpyAsync(l.host, fl.dev + p.off, p.len, hipMemcpyDeviceToHost, l.stream) != hipSuccess ||
            hipStreamSynchronize(l.stream) != hipSuccess)
          e = "D2H failed";
      }
      trace::Span sp("write", "pwrite piece");
      for (uint64_t done = 0; e.empty() && done < p.len;) {
        const ssize_t w = ::pwrite(fl.fd, l.host + done, size_t(p.len - done), off_t(p.off + done));
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) e = std::string("pwrite: ") + std::strerror(errno);
        else done += uint64_t(w);
      }
      if (e.empty()) storage::start_writeback(fl.fd, p.off, p.len);  // the disk works behind the pull
      std::lock_guard<std::mutex> g(mu_);
      if (!e.empty() && fl.err.empty()) fl.err = e;
      --fl.pending;
      --pending_;
      idle_.notify_all();
    }
  }

  size_t piece_;
  std::vector<Lane> lanes_;
  std::vector<std::thread> threads_;
  std::vector<File>* files_ = nullptr;
  std::mutex mu_;
  std::condition_variable work_, idle_;
  std::deque<Piece> q_;
  size_t pending_ = 0;
  bool closing_ = false;
};

// One stats object for the status file: the pipelines' byte and xorb counters summed.
std::string merged_stats(const std::vector<std::unique_ptr<gpurt::DeviceXetPull>>& dps) {
  static const char* keys[] = {"xorbs_from_cache", "xorbs_from_peer", "xorbs_from_cdn", "bytes_from_cache",
                               "bytes_from_peer",  "bytes_from_cdn",  "verify_failures", "refetches"};
  double sum[8] = {0};
  for (auto& d : dps) {
    if (!d) continue;
    const json::Value v = json::Value::parse(d->stats_json());
    for (int i = 0; i < 8; ++i) sum[i] += v[keys[i]].as_double();
  }
  json::Writer w;
  w.obj();
  for (int i = 0; i < 8; ++i) w.key(keys[i]).num_u(uint64_t(sum[i]));
  const double total = sum[3] + sum[4] + sum[5];
  w.key("p2p_ratio").num(total > 0 ? sum[4] / total : 0.0, 4).key("pipelines").num_u(dps.size());
  w.end();
  return w.out();
}

struct Args {
  std::string repo, revision = "main", repo_type = "model";
  std::vector<std::string> peers, dht_bootstrap, include;
  std::optional<std::string> tracker;
  bool p2p = true, dht = true;
  int threads = 16;
  // 256 MiB per staging slot (x 2 slots x 4 pipelines): ample for H2D batches at PCIe speed, and
  // half the pinning of 512 at start-up (8 GB bf16 from a warm seeder: device pulls 1.08 vs 1.40 s,
  // profiles/r5/cli_peer_bf16_st256_r5o.json)
  size_t staging_mb = size_t(std::max(16, env_int("ZEST_GPU_STAGING_MB", 256)));
};

Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    const std::string f = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : std::string(); };
    if (f == "--revision" || f == "-r") a.revision = next();
    else if (f == "--peer" || f == "-p") a.peers.push_back(next());
    else if (f == "--tracker" || f == "-t") a.tracker = next();
    else if (f == "--no-p2p") a.p2p = false;
    else if (f == "--no-dht") a.dht = false;
    else if (f == "--dht-bootstrap") a.dht_bootstrap.push_back(next());
    else if (f == "--repo-type") a.repo_type = next();
    else if (f == "--include") a.include.push_back(next());
    else if (f == "--concurrency" || f == "-j") a.threads = std::max(1, std::atoi(next().c_str()));
    else if (f == "--pipeline-depth") a.staging_mb = size_t(std::max(16, std::atoi(next().c_str())));
    else if (f == "--dht-port" || f == "--listen" || f == "-l") (void)next();  // host-side flags
    else if (!f.empty() && f[0] != '-' && a.repo.empty()) a.repo = f;
    // unknown flags are ignored, like the reference (main.zig:98-119)
  }
  return a;
}

int run(int argc, char** argv) {
  const double t0 = now_s();
  // ZEST_GPU_TRACE=<file.json>: this worker's Chrome trace (ZEST_TRACE would be shared with the CLI)
  if (const char* tp = std::getenv("ZEST_GPU_TRACE"); tp && *tp)
    trace::set_output(std::string(tp) + "." + std::to_string(env_int("ZEST_GPU_RANK", 0)));
  const Args a = parse(argc, argv);
  if (a.repo.empty()) throw Error("Usage", "zest-gpu-worker <repo_id> [pull options]");
  const int rank = env_int("ZEST_GPU_RANK", 0), world = std::max(1, env_int("ZEST_GPU_WORLD", 1));
  const char* status_path = std::getenv("ZEST_GPU_STATUS");
  Config cfg = Config::from_env();
  // HIP runtime start-up and the device pipeline (Xet auth, pinned staging) come up on a side
  // thread while this one lists the repository: both are a few hundred ms on a fresh process.
  // ZEST_GPU_PIPES device pipelines pull different files at the same time, so the write-back
  // always has several files (inodes) to write into at once.
  const int npipes = std::max(1, env_int("ZEST_GPU_PIPES", 4));
  std::vector<std::unique_ptr<gpurt::DeviceXetPull>> dps(static_cast<size_t>(npipes));
  // Write-back: `nwriters` threads, each with its own D2H stream and a pinned piece buffer.
  const int nwriters = std::max(1, env_int("ZEST_GPU_WRITERS", 2 * npipes));
  const size_t piece = size_t(std::max(4, env_int("ZEST_GPU_PIECE_MB", 64))) << 20;
  std::unique_ptr<WriteBack> wb;
  std::string init_err;
  double t_init = 0, t_hip = 0, t_dp = 0;
  std::thread init([&] {
    try {
      // The HIP runtime + device context (~160 ms on a fresh process) come up on their own thread
      // while the pipelines' host halves (xorb cache scan, swarm, Xet auth over HTTP) are built;
      // then every pipeline's pinned staging and the write-back buffers are allocated concurrently.
      std::string hip_err;
      std::thread hip_up([&] {
        try {
          int dev_count = 0;
          hip_ok(hipGetDeviceCount(&dev_count), "hipGetDeviceCount");
          if (dev_count < 1) throw Error("NoDevice", "no GPU visible to this worker");
          hip_ok(hipSetDevice(0), "hipSetDevice");  // the CLI pinned this worker with HIP_VISIBLE_DEVICES
          hip_ok(hipFree(nullptr), "hipFree");      // runtime + device context up
        } catch (const std::exception& e) {
          hip_err = e.what();
        }
        t_hip = now_s();
      });
      struct JoinHip {
        std::thread& t;
        ~JoinHip() {
          if (t.joinable()) t.join();
        }
      } join_hip{hip_up};
      gpurt::DevicePullOptions o;
      o.repo = a.repo;
      o.revision = a.revision;
      o.repo_type = a.repo_type;
      o.p2p = a.p2p;
      o.peers = a.peers;
      o.tracker = a.tracker;
      o.dht = a.dht;
      o.dht_bootstrap = a.dht_bootstrap;
      o.device = 0;
      o.staging_bytes = a.staging_mb << 20;
      o.threads = a.threads;
      o.defer_device = true;
      // One pipeline owns the host state (Xet session, caches, write-behind queue, reconstructions);
      // the others are its siblings: their own streams and pinned staging (2 slots each), no second
      // auth / cache scan (DeviceXetPull::sibling).
      std::vector<std::string> errs(dps.size());
      std::vector<std::thread> mk;
      o.slots = env_int("ZEST_GPU_SLOTS", 2);
      dps[0] = std::make_unique<gpurt::DeviceXetPull>(o);
      for (size_t k = 1; k < dps.size(); ++k) dps[k] = dps[0]->sibling(o.staging_bytes, o.slots);
      hip_up.join();
      if (!hip_err.empty()) throw Error("DeviceInit", hip_err);
      mk.clear();
      for (size_t k = 0; k < dps.size(); ++k)
        mk.emplace_back([&, k] {
          try {
            hip_ok(hipSetDevice(0), "hipSetDevice");
            dps[k]->init_device();
          } catch (const std::exception& e) {
            errs[k] = e.what();
          }
        });
      std::string wb_err;
      try {
        wb = std::make_unique<WriteBack>(nwriters, piece);
      } catch (const std::exception& e) {
        wb_err = e.what();
      }
      for (auto& t : mk) t.join();
      for (auto& e : errs)
        if (!e.empty()) throw Error("DeviceInit", e);
      if (!wb_err.empty()) throw Error("DeviceInit", wb_err);
      t_dp = now_s();
    } catch (const std::exception& e) {
      init_err = e.what();
    }
    t_init = now_s();
  });
  struct Join {
    std::thread& t;
    ~Join() {
      if (t.joinable()) t.join();
    }
  } join_init{init};
  std::optional<trace::Span> phase;
  phase.emplace("worker", "list files");
  std::vector<hub::RepoFile> files = hub::list_files(cfg, a.repo, a.revision, a.repo_type);
  const std::string commit = hub::resolve_commit(cfg, a.repo, a.revision, a.repo_type).value_or(a.revision);
  const std::string snap = cfg.snapshot_dir(a.repo, commit);
  std::vector<hub::RepoFile> xet;
  for (auto& f : files) {
    if (!f.xet_hash) continue;
    bool keep = a.include.empty();
    for (auto& s : a.include)
      keep = keep || (f.path.size() >= s.size() && f.path.compare(f.path.size() - s.size(), s.size(), s) == 0);
    if (keep) xet.push_back(f);
  }
  std::vector<uint64_t> sizes;
  for (auto& f : xet) sizes.push_back(f.size);
  const std::vector<int> owner = assign_owners(sizes, world);
  std::vector<hub::RepoFile> todo;
  size_t cached = 0;
  for (size_t i = 0; i < xet.size(); ++i) {
    if (owner[i] != rank) continue;
    const std::string dst = snap + "/" + xet[i].path;
    bool ok = storage::exists(dst) && storage::file_size(dst) == xet[i].size &&
              (storage::check_verified_marker(cfg, a.repo, commit, xet[i].path, *xet[i].xet_hash, dst) ||
               storage::xet_hash_of_file(dst) == *xet[i].xet_hash);
    if (ok) {
      storage::write_verified_marker(cfg, a.repo, commit, xet[i].path, *xet[i].xet_hash, dst);
      std::cout << "[gpu " << rank << "] " << xet[i].path << " (cached)\n";
      ++cached;
    } else {
      todo.push_back(xet[i]);
    }
  }
  // largest first: the write-back of the file pulled last is the un-overlapped tail
  std::stable_sort(todo.begin(), todo.end(), [](const hub::RepoFile& x, const hub::RepoFile& y) { return x.size > y.size; });
  const double t_list = now_s();
  phase.emplace("worker", "wait device init");
  init.join();
  phase.reset();
  if (!init_err.empty()) throw Error("DeviceInit", init_err);
  const double t_ready = now_s();
  uint64_t done_bytes = 0;
  size_t failed = 0;
  std::string stats = "{}";
  double t_pull = 0, t_write = 0, t_bufs = t_ready, t_last_pull = t_ready, t_last_write = t_ready;
  if (!todo.empty()) {
    // Files go to the device in groups that fit half the free HBM (a 70B repo on one MI355X is one
    // or two groups); each group is ONE pull call -- one pipeline, no drain between files -- and is
    // written back while it is pulled.
    size_t free_b = 0, total_b = 0;
    hip_ok(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    auto padded = [](uint64_t n) { return (n + 4095) / 4096 * 4096; };
    uint64_t max_size = 0;
    for (auto& f : todo) max_size = std::max<uint64_t>(max_size, padded(f.size));
    const uint64_t budget = std::max<uint64_t>(max_size, free_b / 2);
    std::vector<std::pair<size_t, size_t>> groups;  // [begin, end) of todo
    uint64_t gmax = 0;
    for (size_t i = 0; i < todo.size();) {
      uint64_t sum = 0;
      size_t j = i;
      while (j < todo.size() && (j == i || sum + padded(todo[j].size) <= budget)) sum += padded(todo[j++].size);
      groups.emplace_back(i, j);
      gmax = std::max(gmax, sum);
      i = j;
    }
    uint8_t* dbuf = nullptr;
    hip_ok(hipMalloc(reinterpret_cast<void**>(&dbuf), gmax + 4096), "hipMalloc");
    t_bufs = now_s();
    const double tp = now_s();
    for (auto [g0, g1] : groups) {
      std::vector<WriteBack::File> out(g1 - g0);
      std::vector<gpurt::PullRequest> reqs;
      uint64_t off = 0;
      for (size_t i = g0; i < g1; ++i) {
        WriteBack::File& f = out[i - g0];
        f.dst = snap + "/" + todo[i].path;
        f.tmp = f.dst + ".incomplete";
        f.dev = dbuf + off;
        f.size = todo[i].size;
        storage::ensure_dir(f.dst.substr(0, f.dst.rfind('/')));
        f.fd = ::open(f.tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
        if (f.fd < 0) throw Error("IoError", "open " + f.tmp + ": " + std::strerror(errno));
        reqs.push_back({*todo[i].xet_hash, reinterpret_cast<uintptr_t>(f.dev), f.size});
        off += padded(f.size);
      }
      wb->start(&out);
      // deal the group's files to the pipelines, largest first to the least-loaded one
      std::vector<std::vector<size_t>> share(dps.size());
      {
        std::vector<uint64_t> load(dps.size(), 0);
        for (size_t k = 0; k < out.size(); ++k) {
          const size_t p = size_t(std::min_element(load.begin(), load.end()) - load.begin());
          share[p].push_back(k);
          load[p] += out[k].size;
        }
      }
      std::vector<std::string> pipe_err(dps.size());
      std::vector<std::thread> pipes;
      for (size_t p = 0; p < dps.size(); ++p) {
        if (share[p].empty()) continue;
        pipes.emplace_back([&, p] {
          std::vector<gpurt::PullRequest> mine;
          for (size_t k : share[p]) mine.push_back(reqs[k]);
          try {
            dps[p]->pull_files(mine, [&](size_t f, int attempt, uint64_t bytes) {
              wb->progress(share[p][f], attempt, bytes);
            });
          } catch (const std::exception& e) {
            pipe_err[p] = e.what();
          }
          if (!pipe_err[p].empty()) return;
          // This pipeline's files are verified: write what a repair pass replaced, then make them
          // durable now, while the other pipelines are still pulling (not all in the group's tail).
          for (size_t k : share[p])
            if (wb->repaired(k)) wb->post(k, 0, out[k].size);
          wb->wait_files(share[p]);
          for (size_t k : share[p])
            if (out[k].err.empty() && ::fdatasync(out[k].fd) != 0)
              out[k].err = std::string("fdatasync: ") + std::strerror(errno);
        });
      }
      for (auto& t : pipes) t.join();
      std::vector<std::string> file_err(out.size());
      for (size_t p = 0; p < dps.size(); ++p)
        for (size_t k : share[p]) file_err[k] = pipe_err[p];
      t_last_pull = now_s();
      wb->drain();
      wb->stop();
      // (durable before visible: every pipeline fdatasync'ed its files before returning above -- the
      // verified marker trusts size + mtime only, like the host path, downloader.cpp)
      t_last_write = now_s();
      for (size_t k = 0; k < out.size(); ++k) {
        WriteBack::File& f = out[k];
        const hub::RepoFile& rf = todo[g0 + k];
        ::close(f.fd);
        const std::string err = !file_err[k].empty() ? file_err[k] : f.err;
        if (err.empty() && ::rename(f.tmp.c_str(), f.dst.c_str()) == 0) {
          storage::write_verified_marker(cfg, a.repo, commit, rf.path, *rf.xet_hash, f.dst);  // verified on the GPU
          done_bytes += f.size;
          std::cout << "[gpu " << rank << "] " << rf.path << " [xet] " << f.size / 1e6 << " MB verified on the GPU\n";
        } else {
          ::unlink(f.tmp.c_str());
          std::cerr << "[gpu " << rank << "] " << rf.path << ": " << (err.empty() ? "rename failed" : err) << "\n";
          ++failed;
        }
      }
      std::cout << std::flush;
    }
    t_pull = t_last_pull - tp;
    t_write = t_last_write - t_last_pull;  // write-back tail after the last pull call returned
    stats = merged_stats(dps);
  }
  const double dt = now_s() - t0;
  std::cout << "[gpu " << rank << "] " << done_bytes / 1e9 << " GB in " << dt << " s (start " << t_ready - t0
            << " s, device pulls " << t_pull << " s with the write-back streaming behind them, write tail "
            << t_write << " s)\n";
  auto rel = [&](double t) { return std::to_string(int((t - t0) * 1000)); };
  std::cout << "[gpu " << rank << "] timeline ms: listed " << rel(t_list) << ", hip " << rel(t_hip) << ", pipeline "
            << rel(t_dp) << ", device ready " << rel(t_init)
            << ", buffers " << rel(t_bufs) << ", last pull " << rel(t_last_pull) << ", last write "
            << rel(t_last_write) << ", end " << rel(now_s()) << "\n"
            << std::flush;
  if (status_path) {
    json::Writer w;
    w.obj().key("complete").boolean(true).key("rank").num(int64_t(rank)).key("world").num(int64_t(world));
    w.key("failed_files").num_u(failed).key("bytes").num_u(done_bytes).key("files").num_u(todo.size());
    w.key("cached_files").num_u(cached).key("seconds").num(dt, 3).key("pull_s").num(t_pull, 3);
    w.key("write_s").num(t_write, 3).key("init_s").num(t_init - t0, 3).key("list_s").num(t_list - t0, 3);
    // steady-clock instants (CLOCK_MONOTONIC, shared by the processes of one machine): the CLI times
    // this worker's exec + load (spawn -> t0) and stops waiting as soon as this status exists
    w.key("t0_mono").num(t0, 6).key("status_mono").num(now_s(), 6);
    w.key("stats").raw(stats).end();
    storage::write_file_atomic(status_path, w.out() + "\n", true);
  }
  // Every file is written and renamed and the status is on disk: leave without unwinding ~25 GB of
  // device buffers and pinned pieces one free at a time (the OS reclaims them with the process).
  trace::flush();
  std::cout << std::flush;
  std::cerr << std::flush;
  // Let go of the inherited stdout/stderr now: whoever reads them (a shell pipe, a harness waiting
  // for EOF) need not wait for this process's teardown of its device and pinned memory.
  if (const int nul = ::open("/dev/null", O_WRONLY | O_CLOEXEC); nul >= 0) {
    ::dup2(nul, 1);
    ::dup2(nul, 2);
    ::close(nul);
  }
  std::_Exit(failed ? 1 : 0);
}

}  // namespace

int main(int argc, char** argv) {
  try {
    return run(argc, argv);
  } catch (const std::exception& e) {
    std::cerr << "zest-gpu-worker: " << e.what() << "\n";
    return 2;
  }
}
