// `zest` command-line tool: pull / seed / serve / start / stop / status / bench / version / help.
//
// Reference: src/main.zig:40-81 (dispatch), :83-305 (pull), :306-369 (seed), :371-391 (bench),
// :404-468 (serve), :470-503 (start), :552-590 (stop + PID file), :730-776 (usage).  Flags and
// user-visible strings are kept so scripts written against the reference keep working.
// Differences: `seed` keeps serving after announcing (the reference announces and exits,
// main.zig:361-369), re-announcing every `--reannounce` seconds; `serve` can also run a DHT node;
// xorb hashes are parsed with the Xet word-order hex (the reference's seed parses bytewise,
// main.zig:349-356, which yields info-hashes no puller computes).
#include <fcntl.h>
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <iomanip>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <iostream>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "bench.h"
#include "bt_server.h"
#include "config.h"
#include "dht.h"
#include "http.h"
#include "http_api.h"
#include "hub.h"
#include "json.h"
#include "pull.h"
#include "storage.h"
#include "swarm.h"
#include "xet_hash.h"

using namespace zest;

extern char** environ;

namespace {

std::atomic<bool> g_stop{false};
void on_signal(int) { g_stop.store(true); }

std::string self_exe(const char* argv0) {
  char buf[4096];
  ssize_t n = ::readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n > 0) return std::string(buf, size_t(n));
  return argv0;
}

void print_usage(std::ostream& w) {
  w << "zest \xE2\x80\x94 P2P acceleration for ML model distribution (BitTorrent-compliant, AMD Instinct native)\n"
       "\n"
       "Usage:\n"
       "  zest pull <repo_id> [options]    Download a model\n"
       "  zest seed [options]              Seed cached xorbs to peers\n"
       "  zest serve [options]             Run server (BT + HTTP API)\n"
       "  zest start [--open|--no-open]    Start server in background (and open the dashboard)\n"
       "  zest stop                        Stop background server\n"
       "  zest status                      Show background server status\n"
       "  zest bench [options]             Run benchmarks\n"
       "  zest version                     Show version\n"
       "  zest help                        Show this help\n"
       "\n"
       "Pull options:\n"
       "  --revision, -r <ref>     Git revision (default: main)\n"
       "  --peer, -p <ip:port>     Direct peer address (repeatable)\n"
       "  --tracker, -t <url>      BT tracker URL for peer discovery\n"
       "  --dht-port <port>        DHT UDP port (default: 6881)\n"
       "  --dht-bootstrap <h:p>    DHT bootstrap node (repeatable)\n"
       "  --no-dht                 Disable DHT lookups\n"
       "  --listen, -l <addr>      Listen address for P2P (default: 0.0.0.0:6881)\n"
       "  --no-p2p                 Disable P2P, CDN only\n"
       "  --include <suffix>       Only files ending in <suffix> (repeatable)\n"
       "  --concurrency, -j <n>    Parallel term downloads (default: 16)\n"
       "  --no-verify              Skip the Xet file-hash check\n"
       "  --no-serve               Do not auto-start the background seeder\n"
       "  --gpus <n|list>          Decode + verify on n GPUs, or on the listed devices (\"0,2,5\");\n"
       "                           one independent worker per GPU, each pulling its share of the files\n"
       "                           (no collective; for every tensor on every GPU use\n"
       "                           zest_amd.pull(repo, device=\"all\") under torchrun). Default: $ZEST_GPUS\n"
       "  --pipeline-depth <MB>    Pinned staging per GPU worker (default: 1024)\n"
       "\n"
       "Seed options:\n"
       "  --tracker, -t <url>      BT tracker URL\n"
       "  --dht-port <port>        DHT UDP port (default: 6881)\n"
       "  --dht-bootstrap <h:p>    DHT bootstrap node (repeatable)\n"
       "  --listen, -l <addr>      Listen address (default: 0.0.0.0:6881)\n"
       "  --reannounce <sec>       Re-announce interval (default: 900)\n"
       "  --announce-only          Announce and exit (reference behaviour)\n"
       "  --hbm-cache-gb <G>       Upload up to G GB of the xorb cache to GPU memory and seed from it\n"
       "  --device <n>             GPU for --hbm-cache-gb (default: 0)\n"
       "\n"
       "Serve options:\n"
       "  --http-port <port>       HTTP API port (default: 9847)\n"
       "  --listen-port <port>     BT listen port (default: 6881)\n"
       "  --dht                    Also run a DHT node on --dht-port\n"
       "  --fault <spec>           Fault injection, e.g. drop:0.1,corrupt:0.05,delay:20\n"
       "\n"
       "Bench options:\n"
       "  --synthetic              Run synthetic benchmarks\n"
       "  --gpu                    Run the MI355X kernel benchmarks\n"
       "  --json                   Output results as JSON\n"
       "\n"
       "Examples:\n"
       "  zest pull meta-llama/Llama-3.1-8B\n"
       "  zest pull Qwen/Qwen2-7B --revision v1.0 --no-p2p\n"
       "  zest pull gpt2 --peer 10.0.0.5:6881\n"
       "  zest seed --tracker http://tracker.example.com:6881\n"
       "  zest serve --http-port 8080\n"
       "  zest bench --synthetic --json\n";
}

bool parse_port(const std::string& s, uint16_t& out) {
  try {
    int v = std::stoi(s);
    if (v < 0 || v > 65535) return false;
    out = uint16_t(v);
    return true;
  } catch (...) {
    return false;
  }
}

// --listen accepts "port", ":port" or "host:port".
void apply_listen(Config& cfg, const std::string& s) {
  size_t c = s.rfind(':');
  uint16_t p;
  if (parse_port(c == std::string::npos ? s : s.substr(c + 1), p)) cfg.listen_port = p;
}

void write_pid_file(const Config& cfg) {
  try {
    storage::write_file_atomic(cfg.pid_file, std::to_string(::getpid()));
  } catch (const Error&) {
  }
}

std::vector<xet::Hash> cached_xorb_hashes(const Config& cfg) {
  std::set<std::string> uniq;
  for (auto& k : storage::list_cached_xorbs(cfg))
    if (k.size() >= 64) uniq.insert(k.substr(0, 64));
  std::vector<xet::Hash> out;
  for (auto& h : uniq) {
    try {
      out.push_back(xet::from_hex(h));
    } catch (const Error&) {
    }
  }
  return out;
}

int cmd_pull(const std::string& exe, const std::vector<std::string>& a);

// One attempt of `zest pull --gpus N`: N independent worker processes, worker r pinned to
// devices[r] through HIP_VISIBLE_DEVICES.  Files are independent, so there is no rendezvous, no
// torchrun agent and no RCCL communicator: each worker takes its LPT share of the Xet files
// (ZEST_GPU_RANK / ZEST_GPU_WORLD) and writes `{status_base}.{r}` when it ran to the end.  The
// worker is the native `zest-gpu-worker` next to this binary (no Python start-up on the path);
// ZEST_GPU_WORKER_MODULE substitutes `python -m <module>` (tests use a stub).
struct WorkerResult {
  int rc = 0;
  bool complete = false;
  json::Value status;
};

std::vector<WorkerResult> spawn_gpu_workers(const std::string& exe, const std::vector<std::string>& pass,
                                            const std::vector<std::string>& devices, const std::string& status_base) {
  const char* py = std::getenv("ZEST_PYTHON");
  const char* mod = std::getenv("ZEST_GPU_WORKER_MODULE");
  const std::string native = exe.substr(0, exe.rfind('/') + 1) + "zest-gpu-worker";
  std::vector<std::string> base;
  if (mod && *mod) base = {py ? py : "python3", "-m", mod};
  else if (::access(native.c_str(), X_OK) == 0) base = {native};
  else base = {py ? py : "python3", "-m", "zest_amd.multigpu"};
  std::string all;
  for (size_t i = 0; i < devices.size(); ++i) all += (i ? "," : "") + devices[i];
  const int n = int(devices.size());
  std::vector<pid_t> pids(static_cast<size_t>(n), 0);
  std::vector<WorkerResult> out(static_cast<size_t>(n));
  for (int r = 0; r < n; ++r) {
    std::vector<std::string> args = base;
    args.insert(args.end(), pass.begin(), pass.end());
    std::vector<std::string> env_s;
    for (char** e = environ; *e; ++e) {
      const std::string kv = *e;
      const std::string k = kv.substr(0, kv.find('='));
      if (k == "HIP_VISIBLE_DEVICES" || k == "ZEST_GPU_RANK" || k == "ZEST_GPU_WORLD" || k == "ZEST_GPU_STATUS" ||
          k == "ZEST_GPU_DEVICES" || k == "RANK" || k == "WORLD_SIZE" || k == "LOCAL_RANK")
        continue;
      env_s.push_back(kv);
    }
    const std::string st = status_base + "." + std::to_string(r);
    ::unlink(st.c_str());
    env_s.push_back("HIP_VISIBLE_DEVICES=" + devices[size_t(r)]);
    env_s.push_back("ZEST_GPU_RANK=" + std::to_string(r));
    env_s.push_back("ZEST_GPU_WORLD=" + std::to_string(n));
    env_s.push_back("ZEST_GPU_STATUS=" + st);
    env_s.push_back("ZEST_GPU_DEVICES=" + all);
    std::vector<char*> argv, envp;
    for (auto& x : args) argv.push_back(const_cast<char*>(x.c_str()));
    argv.push_back(nullptr);
    for (auto& x : env_s) envp.push_back(const_cast<char*>(x.c_str()));
    envp.push_back(nullptr);
    if (posix_spawnp(&pids[size_t(r)], argv[0], nullptr, nullptr, argv.data(), envp.data()) != 0) {
      std::cerr << "Error: cannot start " << argv[0] << " for --gpus\n";
      pids[size_t(r)] = 0;
      out[size_t(r)].rc = 127;
    }
  }
  // A worker is done when its status file says complete (written after every file is durable and
  // renamed) or when it exits.  The CLI does not wait for a completed worker's exit: tearing down a
  // HIP process (device and pinned allocations) takes a few hundred ms the user need not wait for;
  // the child is reaped with this process.
  auto read_status = [&](int r) -> bool {
    const std::string st = status_base + "." + std::to_string(r);
    auto b = storage::read_file(st);
    if (!b) return false;
    try {
      out[size_t(r)].status = json::Value::parse(std::string(b->begin(), b->end()));
      out[size_t(r)].complete = out[size_t(r)].status["complete"].type() == json::Value::Type::Bool &&
                                out[size_t(r)].status["complete"].as_bool();
    } catch (const Error&) {
      return false;
    }
    return out[size_t(r)].complete;
  };
  const double spawned = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  std::vector<char> done(static_cast<size_t>(n), 0);
  size_t left = 0;
  for (int r = 0; r < n; ++r) left += pids[size_t(r)] ? 1 : 0;
  while (left) {
    for (int r = 0; r < n; ++r) {
      if (!pids[size_t(r)] || done[size_t(r)]) continue;
      int status = 0;
      const pid_t w = ::waitpid(pids[size_t(r)], &status, WNOHANG);
      if (w == pids[size_t(r)]) {
        out[size_t(r)].rc = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
        read_status(r);
      } else if (w == 0 && read_status(r)) {
        out[size_t(r)].rc = out[size_t(r)].status["failed_files"].as_double() > 0 ? 1 : 0;
        const double now = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        const json::Value& s = out[size_t(r)].status;
        if (s["t0_mono"].type() == json::Value::Type::Number)
          std::cout << "[gpu " << r << "] process: exec + load " << int((s["t0_mono"].as_double() - spawned) * 1000)
                    << " ms, run " << int((s["status_mono"].as_double() - s["t0_mono"].as_double()) * 1000)
                    << " ms, status seen after " << int((now - s["status_mono"].as_double()) * 1000)
                    << " ms (exit not awaited)\n" << std::flush;
      } else if (w < 0 && errno == EINTR) {
        continue;
      } else if (w == 0) {
        continue;
      }
      done[size_t(r)] = 1;
      --left;
      ::unlink((status_base + "." + std::to_string(r)).c_str());
    }
    if (left) std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  return out;
}

// `zest pull <repo> --gpus N`: N GPU decode/verify workers, elastic over worker loss.  While the
// workers pull the Xet files, this process fetches the regular files (config, tokenizer) on the
// host.  An attempt in which a worker dies before the end (crash, lost device) is retried on one GPU
// fewer -- the failed devices are dropped first -- and files verified by earlier attempts are
// skipped, so each retry pulls only what is missing; after the single-GPU attempt the host pipeline
// finishes the job (ZEST_GPU_HOST_FALLBACK=0 turns that off).  An attempt whose workers all ran to
// the end but failed files is final: fewer GPUs would not fix the data.  SURVEY §5.3 ("elastic world
// size 8 -> 7"); the reference has no GPU path and no retry (main.zig:233-256).
int pull_on_gpus(const std::string& exe, const std::vector<std::string>& a, int gpus, const std::vector<int>& devices) {
  // exe = <pkg>/_bin/zest -> PYTHONPATH = parent of the package directory (Python workers)
  std::string pkg_parent = exe;
  for (int i = 0; i < 3; ++i) {
    const size_t s = pkg_parent.rfind('/');
    pkg_parent = s == std::string::npos ? "." : pkg_parent.substr(0, s);
  }
  std::string pp = pkg_parent;
  if (const char* old = std::getenv("PYTHONPATH")) pp += std::string(":") + old;
  ::setenv("PYTHONPATH", pp.c_str(), 1);
  std::vector<std::string> pass;
  std::string repo, revision = "main", repo_type = "model";
  bool p2p = true;
  for (size_t i = 0; i < a.size(); ++i) {
    if (a[i] == "--gpus") {
      ++i;
      continue;
    }
    if ((a[i] == "--revision" || a[i] == "-r") && i + 1 < a.size()) revision = a[i + 1];
    if (a[i] == "--repo-type" && i + 1 < a.size()) repo_type = a[i + 1];
    if (a[i] == "--no-p2p") p2p = false;
    if (repo.empty() && !a[i].empty() && a[i][0] != '-' && (i == 0 || a[i - 1].rfind("-", 0) != 0)) repo = a[i];
    pass.push_back(a[i]);
  }
  if (repo.empty()) {
    std::cerr << "Error: missing repository ID\n";
    return 1;
  }
  // Device list: --gpus 0,2,5; else the first N of an inherited HIP_VISIBLE_DEVICES; else 0..N-1.
  std::vector<std::string> devs;
  if (!devices.empty()) {
    for (int d : devices) devs.push_back(std::to_string(d));
  } else {
    std::vector<std::string> vis;
    if (const char* v = std::getenv("HIP_VISIBLE_DEVICES")) {
      std::string s = v;
      for (size_t p = 0; p <= s.size();) {
        size_t e = s.find(',', p);
        if (e == std::string::npos) e = s.size();
        if (e > p) vis.push_back(s.substr(p, e - p));
        p = e + 1;
      }
    }
    for (int i = 0; i < gpus; ++i) devs.push_back(size_t(i) < vis.size() ? vis[size_t(i)] : std::to_string(i));
  }
  Config cfg = Config::from_env();
  std::cout << "zest pull " << repo << " (revision: " << revision << ") on " << devs.size() << " GPU(s)\n" << std::flush;
  // Regular files on the host, concurrently with the GPU workers.
  std::string commit = revision, snap;
  size_t regular_failed = 0, regular_files = 0;
  std::thread host_files([&] {
    try {
      auto files = hub::list_files(cfg, repo, revision, repo_type);
      commit = hub::resolve_commit(cfg, repo, revision, repo_type).value_or(revision);
      snap = cfg.snapshot_dir(repo, commit);
      for (auto& f : files) {
        if (f.xet_hash) continue;
        ++regular_files;
        const std::string dst = snap + "/" + f.path;
        if (storage::exists(dst) && storage::file_size(dst) == f.size) continue;
        try {
          hub::download_regular(cfg, repo, commit, f.path, dst);
        } catch (const Error& e) {
          std::cerr << "  Error downloading " << f.path << ": " << e.what() << "\n";
          ++regular_failed;
        }
      }
    } catch (const Error& e) {
      std::cerr << "  Error listing " << repo << ": " << e.what() << "\n";
      ++regular_failed;
    }
  });
  const char* tmp = std::getenv("TMPDIR");
  const std::string status = std::string(tmp && *tmp ? tmp : "/tmp") + "/zest-gpu-pull-" + std::to_string(::getpid()) +
                             ".json";
  const auto t0 = std::chrono::steady_clock::now();
  int rc = 1;
  bool finished = false;
  std::vector<WorkerResult> res;
  while (!devs.empty()) {
    res = spawn_gpu_workers(exe, pass, devs, status);
    std::vector<std::string> alive, dead;
    for (size_t r = 0; r < res.size(); ++r) (res[r].complete ? alive : dead).push_back(devs[r]);
    if (dead.empty()) {
      finished = true;
      rc = 0;
      for (auto& w : res)
        if (w.rc != 0) rc = w.rc;
      break;
    }
    const size_t n = devs.size();
    std::cerr << "zest: GPU pull on " << n << " GPU(s) stopped before the end (" << dead.size() << " worker(s) lost";
    for (auto& w : res)
      if (!w.complete) std::cerr << ", exit " << w.rc;
    std::cerr << ")";
    if (n > 1) std::cerr << "; retrying on " << n - 1 << " GPU(s), keeping verified files";
    std::cerr << "\n";
    devs = alive;
    devs.insert(devs.end(), dead.begin(), dead.end());
    devs.resize(n - 1);
  }
  host_files.join();
  if (!finished) {
    const char* fb = std::getenv("ZEST_GPU_HOST_FALLBACK");
    if (fb && std::string(fb) == "0") return rc;
    std::cerr << "zest: finishing the pull on the host\n";
    ::unsetenv("ZEST_GPUS");  // the host pass must not start GPU workers again
    return cmd_pull(exe, pass);
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t bytes = 0, failed = regular_failed, peer = 0, cdn = 0, cache = 0;
  for (auto& w : res) {
    bytes += uint64_t(w.status["bytes"].as_double());
    failed += uint64_t(w.status["failed_files"].as_double());
    const json::Value& st = w.status["stats"];
    peer += uint64_t(st["bytes_from_peer"].as_double());
    cdn += uint64_t(st["bytes_from_cdn"].as_double());
    cache += uint64_t(st["bytes_from_cache"].as_double());
  }
  if (!failed) {
    try {
      storage::write_ref(cfg, repo, revision, commit);
    } catch (const Error& e) {
      std::cerr << "Warning: failed to write ref: " << e.what() << "\n";
    }
  }
  const uint64_t src = peer + cdn + cache;
  std::cout << std::fixed << std::setprecision(1);
  std::cout << "\nXorb fetch stats:\n  From peers:   " << peer / 1e6 << " MB\n  From CDN:     " << cdn / 1e6
            << " MB\n  From cache:   " << cache / 1e6 << " MB\n  P2P ratio:    "
            << (src ? 100.0 * double(peer) / double(src) : 0.0) << "%\n";
  std::cout << std::setprecision(2) << "\n" << bytes / 1e9 << " GB verified on " << res.size() << " GPU(s) in " << dt
            << "s (" << (dt > 0 ? bytes / dt / 1e9 : 0.0) << " GB/s)\n";
  std::cout << "\nDone! Model available at:\n  " << snap << "\n" << std::flush;
  if (failed) std::cerr << "zest: " << failed << " file(s) failed\n";
  return failed ? 1 : rc;
}

// `--gpus` value: a count ("4") or a device list ("0,2,5", also "3," for the single device 3).
// Returns the number of GPUs (0 = host path) and fills `devices` for a list.
int parse_gpus(const std::string& v, std::vector<int>& devices) {
  devices.clear();
  if (v.find(',') == std::string::npos) return std::max(0, std::atoi(v.c_str()));
  size_t s = 0;
  while (s < v.size()) {
    size_t e = v.find(',', s);
    if (e == std::string::npos) e = v.size();
    const std::string tok = v.substr(s, e - s);
    if (!tok.empty()) {
      if (tok.find_first_not_of("0123456789") != std::string::npos) return 0;
      devices.push_back(std::atoi(tok.c_str()));
    }
    s = e + 1;
  }
  return int(devices.size());
}

int cmd_pull(const std::string& exe, const std::vector<std::string>& a) {
  std::string gpus_arg;
  for (size_t i = 0; i + 1 < a.size(); ++i)
    if (a[i] == "--gpus") gpus_arg = a[i + 1];
  if (gpus_arg.empty())
    if (const char* g = std::getenv("ZEST_GPUS")) gpus_arg = g;
  if (!gpus_arg.empty()) {
    std::vector<int> devices;
    const int n = parse_gpus(gpus_arg, devices);
    if (n > 0) return pull_on_gpus(exe, a, n, devices);
  }
  if (a.empty() || a[0].rfind("-", 0) == 0) {
    std::cerr << "Error: missing repository ID\n"
              << "Usage: zest pull <repo_id> [--revision <ref>] [--tracker <url>] [--no-p2p]\n";
    return 1;
  }
  Config cfg = Config::from_env();
  PullOptions o;
  o.repo_id = a[0];
  for (size_t i = 1; i < a.size(); ++i) {
    const std::string& f = a[i];
    auto next = [&]() -> std::string { return i + 1 < a.size() ? a[++i] : std::string(); };
    if (f == "--revision" || f == "-r") o.revision = next();
    else if (f == "--tracker" || f == "-t") o.tracker = next();
    else if (f == "--peer" || f == "-p") o.peers.push_back(next());
    else if (f == "--dht-port") parse_port(next(), cfg.dht_port);
    else if (f == "--dht-bootstrap") o.dht_bootstrap.push_back(next());
    else if (f == "--no-dht") o.dht = false;
    else if (f == "--listen" || f == "-l") apply_listen(cfg, next());
    else if (f == "--no-p2p") o.p2p = false;
    else if (f == "--include") o.include.push_back(next());
    else if (f == "--concurrency" || f == "-j") o.concurrency = std::atoi(next().c_str());
    else if (f == "--no-verify") o.verify = false;
    else if (f == "--no-serve") o.autostart_server = false;
    else if (f == "--repo-type") o.repo_type = next();
    else std::cerr << "Warning: unknown option " << f << "\n";
  }
  try {
    PullSummary s = run_pull(cfg, o, std::cout, std::cerr);
    if (o.p2p && o.autostart_server && !std::getenv("ZEST_NO_AUTOSTART")) {
      if (!server_healthy(cfg.http_port, 300) && spawn_background_server(exe, cfg.http_port)) {
        std::cout << "Seeding in background (BT :" << cfg.listen_port << ", HTTP :" << cfg.http_port << ")\n";
        std::cout << "Dashboard: http://localhost:" << cfg.http_port << "\n";
      }
    }
    (void)s;
    return 0;
  } catch (const Error& e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
}

// `zest seed --hbm-cache-gb G [--device N]`: seed from GPU memory — the disk xorb cache is uploaded
// to HBM and served by the HBM seeder (`python -m zest_amd.seed`, csrc/bind/hip_seed.cpp), run as a
// child process of this CLI.
int seed_from_hbm(const std::string& exe, const Config& cfg, const std::string& gb, const std::string& device) {
  std::string pkg_parent = exe;
  for (int i = 0; i < 3; ++i) {
    const size_t s = pkg_parent.rfind('/');
    pkg_parent = s == std::string::npos ? "." : pkg_parent.substr(0, s);
  }
  std::string pp = pkg_parent;
  if (const char* old = std::getenv("PYTHONPATH")) pp += std::string(":") + old;
  ::setenv("PYTHONPATH", pp.c_str(), 1);
  const char* py = std::getenv("ZEST_PYTHON");
  const char* mod = std::getenv("ZEST_SEED_MODULE");  // tests substitute a stub
  std::vector<std::string> args = {py ? py : "python3", "-m", mod && *mod ? mod : "zest_amd.seed",
                                   "--port", std::to_string(cfg.listen_port), "--device", "cuda:" + device,
                                   "--max-gb", gb};
  std::vector<char*> argv;
  for (auto& s : args) argv.push_back(const_cast<char*>(s.c_str()));
  argv.push_back(nullptr);
  pid_t pid = 0;
  if (posix_spawnp(&pid, argv[0], nullptr, nullptr, argv.data(), environ) != 0) {
    std::cerr << "Error: cannot start " << argv[0] << " for --hbm-cache-gb\n";
    return 127;
  }
  int status = 0;
  while (::waitpid(pid, &status, 0) < 0 && errno == EINTR) {
  }
  return WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
}

int cmd_seed(const std::string& exe, const std::vector<std::string>& a) {
  Config cfg = Config::from_env();
  std::string hbm_gb, hbm_dev = "0";
  std::optional<std::string> tracker;
  std::vector<net::Addr> boot;
  int reannounce = 900;
  bool announce_only = false;
  for (size_t i = 0; i < a.size(); ++i) {
    const std::string& f = a[i];
    auto next = [&]() -> std::string { return i + 1 < a.size() ? a[++i] : std::string(); };
    if (f == "--tracker" || f == "-t") tracker = next();
    else if (f == "--listen" || f == "-l") apply_listen(cfg, next());
    else if (f == "--dht-port") parse_port(next(), cfg.dht_port);
    else if (f == "--dht-bootstrap") {
      try {
        boot.push_back(net::Addr::parse(next(), 6881));
      } catch (const Error&) {
      }
    } else if (f == "--reannounce") reannounce = std::max(5, std::atoi(next().c_str()));
    else if (f == "--announce-only") announce_only = true;
    else if (f == "--hbm-cache-gb") hbm_gb = next();
    else if (f == "--device") hbm_dev = next();
  }
  if (!hbm_gb.empty()) return seed_from_hbm(exe, cfg, hbm_gb, hbm_dev);
  std::cout << "Scanning local xorb cache...\n";
  auto hashes = cached_xorb_hashes(cfg);
  std::cout << "Found " << hashes.size() << " cached xorbs\n";
  if (hashes.empty()) {
    std::cout << "Nothing to seed. Run `zest pull` first.\n";
    return 0;
  }
  storage::XorbRegistry registry;
  registry.scan(cfg);
  storage::XorbCache cache(cfg, &registry);
  std::unique_ptr<bt::BtServer> server;
  if (!announce_only) {
    try {
      server = std::make_unique<bt::BtServer>(cfg, &cache, bt::PieceProvider{}, cfg.listen_port);
      if (!cfg.fault.empty()) server->set_fault(bt::FaultSpec::parse(cfg.fault));
      server->start();
      cfg.listen_port = server->port();
    } catch (const Error& e) {
      std::cerr << "Error: cannot listen on port " << cfg.listen_port << " (" << e.what() << ")\n";
      return 1;
    }
  }
  SwarmDownloader swarm(cfg, tracker, true, true, boot);
  // default routers bootstrap in the background: give them a bounded moment before announcing
  for (int i = 0; i < 500 && !swarm.bootstrap_done(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  swarm.announce(hashes);
  std::cout << "Announced " << hashes.size() << " xorbs via BT protocol\n";
  std::cout << "  Peer ID: " << peer_id::kClientPrefix << "...\n";
  std::cout << "  DHT port: " << cfg.dht_port << "\n";
  std::cout << "  Listen port: " << cfg.listen_port << "\n";
  if (tracker) std::cout << "  Tracker: " << *tracker << "\n";
  std::cout << "Seeding...\n" << std::flush;
  if (announce_only) return 0;
  ::signal(SIGINT, on_signal);
  ::signal(SIGTERM, on_signal);
  auto last = std::chrono::steady_clock::now();
  while (!g_stop.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    if (std::chrono::steady_clock::now() - last > std::chrono::seconds(reannounce)) {
      swarm.announce(cached_xorb_hashes(cfg));
      last = std::chrono::steady_clock::now();
    }
  }
  server->stop();
  auto st = server->stats();
  std::cout << "\nSeeding stopped. Served " << st.chunks_served << " chunk ranges (" << st.bytes_served
            << " bytes) to " << st.total_peers << " peers.\n";
  return 0;
}

// `python -m <module> <args>` as a child process of this CLI (the package directory next to the
// binary on PYTHONPATH); returns its exit code.  The CLI never initialises the GPU itself.
int run_python_module(const std::string& exe, const std::string& module, const std::vector<std::string>& extra) {
  std::string pkg_parent = exe;  // <pkg_parent>/zest_amd/_bin/zest
  for (int i = 0; i < 3; ++i) {
    const size_t s = pkg_parent.rfind('/');
    pkg_parent = s == std::string::npos ? "." : pkg_parent.substr(0, s);
  }
  std::string pp = pkg_parent;
  if (const char* old = std::getenv("PYTHONPATH")) pp += std::string(":") + old;
  ::setenv("PYTHONPATH", pp.c_str(), 1);
  const char* py = std::getenv("ZEST_PYTHON");
  std::vector<std::string> args = {py ? py : "python3", "-m", module};
  args.insert(args.end(), extra.begin(), extra.end());
  std::vector<char*> argv;
  for (auto& s : args) argv.push_back(const_cast<char*>(s.c_str()));
  argv.push_back(nullptr);
  pid_t pid = 0;
  if (posix_spawnp(&pid, argv[0], nullptr, nullptr, argv.data(), environ) != 0) {
    std::cerr << "Error: cannot start " << argv[0] << " -m " << module << "\n";
    return 127;
  }
  int status = 0;
  while (::waitpid(pid, &status, 0) < 0 && errno == EINTR) {
  }
  return WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
}

int cmd_bench(const std::string& exe, const std::vector<std::string>& a) {
  bool json = false, synthetic = false, core_only = false, gpu = false;
  for (auto& f : a) {
    if (f == "--json") json = true;
    else if (f == "--synthetic") synthetic = true;
    else if (f == "--core") core_only = true;
    else if (f == "--gpu") gpu = true;
  }
  if (gpu) {  // device rows (K1-K6 kernels, H2D), same JSON schema: zest_amd/gpubench.py
    std::vector<std::string> extra;
    if (json) extra.push_back("--json");
    return run_python_module(exe, "zest_amd.gpubench", extra);
  }
  if (!synthetic) {
    std::cerr << "Usage: zest bench --synthetic [--json]\n"
              << "  --synthetic  Run bencode/hash/wire benchmarks\n"
              << "  --json       Output results as JSON\n"
              << "  --core       Only the five reference rows\n"
              << "  --gpu        MI355X kernel rows (BLAKE3, SHA-1, CDC, xorb verify, LZ4/BG4, Merkle, H2D)\n";
    return 0;
  }
  auto r = bench::run_synthetic(!core_only);
  if (json) bench::write_json(std::cout, r);
  else bench::write_text(std::cout, r);
  return 0;
}

int cmd_serve(const std::vector<std::string>& a) {
  Config cfg = Config::from_env();
  bool run_dht = false;
  std::vector<net::Addr> boot;
  for (size_t i = 0; i < a.size(); ++i) {
    const std::string& f = a[i];
    auto next = [&]() -> std::string { return i + 1 < a.size() ? a[++i] : std::string(); };
    if (f == "--http-port") parse_port(next(), cfg.http_port);
    else if (f == "--listen-port") parse_port(next(), cfg.listen_port);
    else if (f == "--dht") run_dht = true;
    else if (f == "--dht-port") parse_port(next(), cfg.dht_port);
    else if (f == "--dht-bootstrap") {
      try {
        boot.push_back(net::Addr::parse(next(), 6881));
      } catch (const Error&) {
      }
    } else if (f == "--fault") cfg.fault = next();
  }
  storage::XorbRegistry registry;
  registry.scan(cfg);
  storage::XorbCache cache(cfg, &registry);
  std::unique_ptr<bt::BtServer> bt;
  try {
    bt = std::make_unique<bt::BtServer>(cfg, &cache, bt::PieceProvider{}, cfg.listen_port);
    if (!cfg.fault.empty()) bt->set_fault(bt::FaultSpec::parse(cfg.fault));
  } catch (const Error& e) {
    std::cerr << "Error: BT listen failed on port " << cfg.listen_port << ": " << e.what() << "\n";
    return 1;
  }
  std::unique_ptr<ApiServer> api;
  try {
    api = std::make_unique<ApiServer>(cfg, bt.get(), &registry, "");
  } catch (const Error& e) {
    std::cerr << "HTTP API error: " << e.what() << "\n";
    return 1;
  }
  std::cout << "zest server v" << kVersion << "\n";
  std::cout << "  BT listen port: " << bt->port() << "\n";
  std::cout << "  HTTP API port:  " << api->port() << "\n";
  std::cout << "  Peer ID:        " << peer_id::kClientPrefix << "...\n";
  std::cout << "  Cached xorbs:   " << registry.count() << "\n";
  std::unique_ptr<dht::Dht> node;
  if (run_dht) {
    node = std::make_unique<dht::Dht>(cfg.dht_port);
    node->start();
    if (boot.empty())  // default public routers, each resolved with a deadline (offline: skipped)
      for (const std::string& r : cfg.dht_routers)
        if (auto ra = net::resolve_with_deadline(r, 6881, 1500)) boot.push_back(*ra);
    if (!boot.empty()) node->bootstrap(boot, 1500);
    std::cout << "  DHT port:       " << node->port() << "\n";
  }
  std::cout << "\nServer running. Press Ctrl+C to stop.\n" << std::flush;
  write_pid_file(cfg);
  ::signal(SIGINT, on_signal);
  ::signal(SIGTERM, on_signal);
  ::signal(SIGPIPE, SIG_IGN);
  bt->start();
  api->start();
  auto last_announce = std::chrono::steady_clock::now() - std::chrono::hours(1);
  while (!g_stop.load() && !api->stopping()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (node && std::chrono::steady_clock::now() - last_announce > std::chrono::minutes(15)) {
      for (auto& h : cached_xorb_hashes(cfg)) node->announce_peer(peer_id::info_hash(h.data()), bt->port(), 1000);
      last_announce = std::chrono::steady_clock::now();
    }
  }
  api->stop();
  bt->stop();
  if (node) node->stop();
  api.reset();
  storage::remove_file(cfg.pid_file);
  std::cout << "\nServer stopped.\n";
  return 0;
}

// Open the dashboard in a browser (xdg-open / open), detached; false when no opener could start.
bool open_dashboard(const std::string& url) {
#ifdef __APPLE__
  const char* opener = "open";
#else
  const char* opener = "xdg-open";
#endif
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_addopen(&fa, 1, "/dev/null", O_WRONLY, 0);
  posix_spawn_file_actions_addopen(&fa, 2, "/dev/null", O_WRONLY, 0);
  const char* argv[] = {opener, url.c_str(), nullptr};
  pid_t pid = 0;
  const int rc = posix_spawnp(&pid, opener, &fa, nullptr, const_cast<char* const*>(argv), environ);
  posix_spawn_file_actions_destroy(&fa);
  return rc == 0;
}

// `zest start [--open | --no-open]`: start the background server.  The reference always runs
// xdg-open/open on the dashboard (main.zig:485-529); here that happens only with --open, or by
// default when a desktop session is present (DISPLAY / WAYLAND_DISPLAY), so headless GPU servers
// never try to launch a browser.  ZEST_OPEN_DASHBOARD=0/1 sets the default.
int cmd_start(const std::string& exe, const std::vector<std::string>& a) {
  Config cfg = Config::from_env();
  auto set = [](const char* k) {
    const char* v = std::getenv(k);
    return v && *v;
  };
  bool open = set("DISPLAY") || set("WAYLAND_DISPLAY");
  if (const char* e = std::getenv("ZEST_OPEN_DASHBOARD")) open = std::string(e) == "1";
  for (auto& f : a) {
    if (f == "--open") open = true;
    else if (f == "--no-open") open = false;
  }
  const std::string url = "http://localhost:" + std::to_string(cfg.http_port);
  if (server_healthy(cfg.http_port, 500)) {
    std::cerr << "zest server is already running on port " << cfg.http_port << ".\n";
    if (open && !open_dashboard(url)) std::cerr << "Could not open a browser; dashboard: " << url << "\n";
    return 0;
  }
  if (!spawn_background_server(exe, cfg.http_port)) {
    std::cerr << "Failed to start zest server.\n";
    return 1;
  }
  for (int i = 0; i < 50 && !server_healthy(cfg.http_port, 200); ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  std::cout << "Seeding in background (BT :" << cfg.listen_port << ", HTTP :" << cfg.http_port << ")\n";
  std::cout << "Dashboard: " << url << "\n";
  if (open) {
    if (open_dashboard(url)) std::cout << "Opened the dashboard in a browser\n";
    else std::cerr << "Could not open a browser (no xdg-open); dashboard: " << url << "\n";
  }
  return 0;
}

int cmd_stop() {
  Config cfg = Config::from_env();
  auto pid = storage::read_file(cfg.pid_file);
  std::string pid_str = pid ? std::string(pid->begin(), pid->end()) : "";
  while (!pid_str.empty() && std::isspace(uint8_t(pid_str.back()))) pid_str.pop_back();
  if (pid_str.empty()) {
    std::cerr << "No running zest server found.\n";
    return 1;
  }
  try {
    http::RequestOptions ro;
    ro.timeout_ms = 3000;
    auto r = http::request("POST", "http://127.0.0.1:" + std::to_string(cfg.http_port) + "/v1/stop", {}, "", ro);
    if (r.status == 200) {
      std::cout << "zest server stopped (was PID " << pid_str << ").\n";
      return 0;
    }
    std::cerr << "Server returned status " << r.status << ".\n";
    return 1;
  } catch (const Error&) {
    std::cerr << "Failed to connect to zest server. It may have already stopped.\n";
    storage::remove_file(cfg.pid_file);
    return 1;
  }
}

int cmd_status() {
  Config cfg = Config::from_env();
  try {
    http::RequestOptions ro;
    ro.timeout_ms = 2000;
    auto r = http::get("http://127.0.0.1:" + std::to_string(cfg.http_port) + "/v1/status", {}, ro);
    std::cout << std::string(r.body.begin(), r.body.end()) << "\n";
    return r.status == 200 ? 0 : 1;
  } catch (const Error&) {
    std::cerr << "No running zest server found.\n";
    return 1;
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::ios::sync_with_stdio(true);
  const std::string exe = self_exe(argv[0]);
  if (argc < 2) {
    print_usage(std::cout);
    return 0;
  }
  const std::string cmd = argv[1];
  std::vector<std::string> rest(argv + 2, argv + argc);
  try {
    if (cmd == "pull") return cmd_pull(exe, rest);
    if (cmd == "seed") return cmd_seed(exe, rest);
    if (cmd == "bench") return cmd_bench(exe, rest);
    if (cmd == "serve") return cmd_serve(rest);
    if (cmd == "start") return cmd_start(exe, rest);
    if (cmd == "stop") return cmd_stop();
    if (cmd == "status") return cmd_status();
    if (cmd == "version" || cmd == "--version" || cmd == "-V") {
      std::cout << "zest " << kVersion << "\n";
      return 0;
    }
    if (cmd == "help" || cmd == "--help" || cmd == "-h") {
      print_usage(std::cout);
      return 0;
    }
    std::cerr << "Unknown command: " << cmd << "\n\n";
    print_usage(std::cout);
    return 1;
  } catch (const std::exception& e) {
    std::cerr << "Error: " << e.what() << "\n";
    return 1;
  }
}
