// `zest-gpu-worker`: one process per GPU for `zest pull <repo> --gpus N` (started by the CLI with
// HIP_VISIBLE_DEVICES pinned to one device).  Native end to end -- no Python or torch start-up on
// the path, no torchrun agent and no RCCL communicator (files are independent, so the workers never
// talk to each other; the CLI aggregates their status files).
//
//   list files (Hub API) -> this worker's Xet files (LPT by size over ZEST_GPU_WORLD workers)
//   -> skip verified cached files -> device-direct pull (DeviceXetPull: fetch -> pinned -> H2D ->
//   GPU decode + BLAKE3 + Merkle verify into HBM) -> snapshot write-back (D2H in 256 MiB pieces
//   into pinned slots on a side stream, pwrite threads), overlapped with the next file's pull.
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
#include <string>
#include <thread>
#include <vector>

#include "config.h"
#include "device_pull.h"
#include "hub.h"
#include "json.h"
#include "storage.h"

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

// Device buffer -> file: D2H of piece k+1 (side stream, pinned slot) overlaps the pwrite of piece k
// (`writers` threads).  The snapshot write is the slow leg of a GPU pull (page cache), so it runs on
// several threads and overlaps the next file's device pull.
class Writer {
 public:
  Writer(size_t piece, int slots) : piece_(piece) {
    hip_ok(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    slots_.resize(size_t(slots));
    for (auto& s : slots_) {
      hip_ok(hipHostMalloc(reinterpret_cast<void**>(&s.host), piece_, hipHostMallocDefault), "hipHostMalloc");
      hip_ok(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming), "hipEventCreate");
    }
  }
  ~Writer() {
    (void)hipStreamSynchronize(stream_);
    for (auto& s : slots_) {
      if (s.host) (void)hipHostFree(s.host);
      if (s.ev) (void)hipEventDestroy(s.ev);
    }
    (void)hipStreamDestroy(stream_);
  }

  // ZEST_GPU_ODIRECT=1: whole 4 KiB-multiple pieces go to the file with O_DIRECT straight from the
  // pinned slot (DMA, no CPU copy into the page cache; the tail piece is written buffered).
  void write(const uint8_t* dev, uint64_t n, const std::string& path) {
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) throw Error("IoError", "open " + path + ": " + std::strerror(errno));
    int dfd = -1;
    if (env_int("ZEST_GPU_ODIRECT", 0) == 1) dfd = ::open(path.c_str(), O_WRONLY | O_DIRECT | O_CLOEXEC);
    std::string err;
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int> busy(slots_.size(), 0);
    bool failed = false;
    for (uint64_t off = 0, k = 0; off < n && !failed; off += piece_, ++k) {
      const size_t s = size_t(k % slots_.size());
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return !busy[s] || failed; });
        if (failed) break;
        busy[s] = 1;
      }
      const uint64_t m = std::min<uint64_t>(piece_, n - off);
      hip_ok(hipMemcpyAsync(slots_[s].host, dev + off, m, hipMemcpyDeviceToHost, stream_), "D2H");
      hip_ok(hipEventRecord(slots_[s].ev, stream_), "event");
      th.emplace_back([&, s, m, off] {
        std::string e;
        if (hipEventSynchronize(slots_[s].ev) != hipSuccess) e = "D2H failed";
        const int wfd = (dfd >= 0 && m % 4096 == 0 && off % 4096 == 0) ? dfd : fd;
        for (uint64_t done = 0; e.empty() && done < m;) {
          const ssize_t w = ::pwrite(wfd, slots_[s].host + done, size_t(m - done), off_t(off + done));
          if (w < 0 && errno == EINTR) continue;
          if (w <= 0) e = std::string("pwrite: ") + std::strerror(errno);
          else done += uint64_t(w);
        }
        std::lock_guard<std::mutex> g(mu);
        if (!e.empty() && err.empty()) err = e, failed = true;
        busy[s] = 0;
        cv.notify_all();
      });
    }
    for (auto& t : th) t.join();
    if (dfd >= 0) ::close(dfd);
    ::close(fd);
    if (!err.empty()) throw Error("IoError", path + ": " + err);
  }

 private:
  struct Slot {
    uint8_t* host = nullptr;
    hipEvent_t ev = nullptr;
  };
  size_t piece_;
  hipStream_t stream_ = nullptr;
  std::vector<Slot> slots_;
};

struct Args {
  std::string repo, revision = "main", repo_type = "model";
  std::vector<std::string> peers, dht_bootstrap, include;
  std::optional<std::string> tracker;
  bool p2p = true, dht = true;
  int threads = 16;
  size_t staging_mb = 1024;
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
  const Args a = parse(argc, argv);
  if (a.repo.empty()) throw Error("Usage", "zest-gpu-worker <repo_id> [pull options]");
  const int rank = env_int("ZEST_GPU_RANK", 0), world = std::max(1, env_int("ZEST_GPU_WORLD", 1));
  const char* status_path = std::getenv("ZEST_GPU_STATUS");
  Config cfg = Config::from_env();
  // HIP runtime start-up and the device pipeline (Xet auth, pinned staging) come up on a side
  // thread while this one lists the repository: both are a few hundred ms on a fresh process.
  std::unique_ptr<gpurt::DeviceXetPull> dp;
  std::string init_err;
  double t_init = 0;
  std::thread init([&] {
    try {
      int dev_count = 0;
      hip_ok(hipGetDeviceCount(&dev_count), "hipGetDeviceCount");
      if (dev_count < 1) throw Error("NoDevice", "no GPU visible to this worker");
      hip_ok(hipSetDevice(0), "hipSetDevice");  // the CLI pinned this worker with HIP_VISIBLE_DEVICES
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
      dp = std::make_unique<gpurt::DeviceXetPull>(o);
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
  init.join();
  if (!init_err.empty()) throw Error("DeviceInit", init_err);
  const double t_ready = now_s();
  uint64_t done_bytes = 0;
  size_t failed = 0;
  std::string stats = "{}";
  double t_pull = 0, t_write = 0, t_bufs = t_ready, t_last_pull = t_ready, t_last_write = t_ready;
  if (!todo.empty()) {
    uint64_t max_size = 1;
    for (auto& f : todo) max_size = std::max(max_size, f.size);
    // Device buffer pool: file i is pulled into a free buffer while earlier files are written back
    // by `nwriters` threads, each on a different file (concurrent pwrites to ONE file serialize on
    // its inode; the host pull writes 4 files at once for the same reason).  As many buffers as
    // half the free HBM holds, capped by the file count: a 70B repo (30 x 4.7 GB) fits whole.
    size_t free_b = 0, total_b = 0;
    hip_ok(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    const size_t nbuf = std::max<size_t>(2, std::min<size_t>(todo.size(), (free_b / 2) / (max_size + 4096)));
    const int nwriters = int(std::min<size_t>(size_t(std::max(1, env_int("ZEST_GPU_WRITERS", 2))), todo.size()));
    const int wslots = std::max(2, env_int("ZEST_GPU_WRITE_SLOTS", 3));
    std::vector<uint8_t*> bufs(std::min(nbuf, todo.size()), nullptr);
    for (auto& bp : bufs) hip_ok(hipMalloc(reinterpret_cast<void**>(&bp), max_size + 4096), "hipMalloc");
    t_bufs = now_s();
    std::vector<int> free_bufs;
    for (int k = int(bufs.size()) - 1; k >= 0; --k) free_bufs.push_back(k);
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<size_t, int>> queue;  // (file, buffer) verified in HBM, waiting for write-back
    bool closing = false;
    auto write_loop = [&] {
      Writer writer(size_t(256) << 20, wslots);  // own D2H stream + pinned slots per writer thread
      while (true) {
        std::pair<size_t, int> job;
        {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [&] { return closing || !queue.empty(); });
          if (queue.empty()) return;
          job = queue.front();
          queue.pop_front();
        }
        const hub::RepoFile& f = todo[job.first];
        const std::string dst = snap + "/" + f.path;
        const double tw = now_s();
        try {
          const size_t slash = dst.rfind('/');
          storage::ensure_dir(dst.substr(0, slash));
          writer.write(bufs[size_t(job.second)], f.size, dst + ".incomplete");
          if (::rename((dst + ".incomplete").c_str(), dst.c_str()) != 0) throw Error("IoError", "rename " + dst);
          storage::write_verified_marker(cfg, a.repo, commit, f.path, *f.xet_hash, dst);  // verified on the GPU
          std::lock_guard<std::mutex> g(mu);
          done_bytes += f.size;
          t_last_write = now_s();
          t_write += t_last_write - tw;
          std::cout << "[gpu " << rank << "] " << f.path << " [xet] " << f.size / 1e6 << " MB verified on the GPU\n"
                    << std::flush;
        } catch (const std::exception& e) {
          std::lock_guard<std::mutex> g(mu);
          std::cerr << "[gpu " << rank << "] " << f.path << ": write failed: " << e.what() << "\n";
          ++failed;
        }
        std::lock_guard<std::mutex> g(mu);
        free_bufs.push_back(job.second);
        cv.notify_all();
      }
    };
    // ZEST_GPU_WRITE_AFTER=1: write back only after every pull finished (needs a buffer per file;
    // measures the two legs separately).
    const bool write_after = env_int("ZEST_GPU_WRITE_AFTER", 0) == 1 && bufs.size() >= todo.size();
    std::vector<std::thread> writers;
    if (!write_after)
      for (int w = 0; w < nwriters; ++w) writers.emplace_back(write_loop);
    const double tp = now_s();
    for (size_t i = 0; i < todo.size(); ++i) {
      int b;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return !free_bufs.empty(); });
        b = free_bufs.back();
        free_bufs.pop_back();
      }
      try {
        dp->pull_files({{*todo[i].xet_hash, reinterpret_cast<uintptr_t>(bufs[size_t(b)]), todo[i].size}});
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu);
        std::cerr << "[gpu " << rank << "] " << todo[i].path << ": error " << e.what() << "\n";
        ++failed;
        free_bufs.push_back(b);
        continue;
      }
      std::lock_guard<std::mutex> g(mu);
      t_last_pull = now_s();
      queue.emplace_back(i, b);
      cv.notify_all();
    }
    t_pull = now_s() - tp;
    if (write_after)
      for (int w = 0; w < nwriters; ++w) writers.emplace_back(write_loop);
    {
      std::lock_guard<std::mutex> g(mu);
      closing = true;
      cv.notify_all();
    }
    for (auto& t : writers) t.join();
    for (auto& bp : bufs) (void)hipFree(bp);
    stats = dp->stats_json();
  }
  const double dt = now_s() - t0;
  std::cout << "[gpu " << rank << "] " << done_bytes / 1e9 << " GB in " << dt << " s (start " << t_ready - t0
            << " s, device pulls " << t_pull << " s, writes " << t_write << " s summed over writer threads, "
            << "overlapped)\n";
  auto rel = [&](double t) { return std::to_string(int((t - t0) * 1000)); };
  std::cout << "[gpu " << rank << "] timeline ms: listed " << rel(t_list) << ", device ready " << rel(t_init)
            << ", buffers " << rel(t_bufs) << ", last pull " << rel(t_last_pull) << ", last write "
            << rel(t_last_write) << ", end " << rel(now_s()) << "\n"
            << std::flush;
  if (status_path) {
    json::Writer w;
    w.obj().key("complete").boolean(true).key("rank").num(int64_t(rank)).key("world").num(int64_t(world));
    w.key("failed_files").num_u(failed).key("bytes").num_u(done_bytes).key("files").num_u(todo.size());
    w.key("cached_files").num_u(cached).key("seconds").num(dt, 3).key("pull_s").num(t_pull, 3);
    w.key("write_s").num(t_write, 3).key("init_s").num(t_init - t0, 3).key("list_s").num(t_list - t0, 3);
    w.key("stats").raw(stats).end();
    storage::write_file_atomic(status_path, w.out() + "\n", true);
  }
  return failed ? 1 : 0;
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
