#include "trace.h"

#include <dlfcn.h>

#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "json.h"

namespace zest::trace {

namespace {

struct State {
  std::mutex mu;
  std::atomic<int> mode{-1};
  std::string path;
  std::vector<std::string> events;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  bool atexit_registered = false;
};

State& st() {
  static State* s = new State();  // leaked on purpose: usable from atexit and late threads
  return *s;
}

uint32_t tid() { return uint32_t(::syscall(SYS_gettid)); }

void at_exit() { flush(); }

void init_locked(State& s, const char* v) {
  if (!v || !*v || std::strcmp(v, "0") == 0) {
    s.mode.store(kOff);
    return;
  }
  if (std::strcmp(v, "1") == 0 || std::strcmp(v, "log") == 0) {
    s.mode.store(kLog);
    return;
  }
  s.path = v;
  // "%p" in the path: this process's pid (several processes tracing at once, e.g. a swarm's ranks
  // and the seeder they pull from)
  if (const size_t k = s.path.find("%p"); k != std::string::npos) s.path.replace(k, 2, std::to_string(::getpid()));
  s.mode.store(kFile);
  if (!s.atexit_registered) {
    std::atexit(at_exit);
    s.atexit_registered = true;
  }
}

}  // namespace

namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  bool on = false;
};

const Roctx& roctx() {
  static const Roctx r = [] {
    Roctx x;
    const char* e = std::getenv("ZEST_ROCTX");
    if (!e || !*e || *e == '0') return x;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"}) {
      if (void* h = ::dlopen(lib, RTLD_NOW | RTLD_GLOBAL)) {
        x.push = reinterpret_cast<int (*)(const char*)>(::dlsym(h, "roctxRangePushA"));
        x.pop = reinterpret_cast<int (*)()>(::dlsym(h, "roctxRangePop"));
        if (x.push && x.pop) break;
      }
    }
    x.on = x.push && x.pop;
    return x;
  }();
  return r;
}
}  // namespace

bool roctx_enabled() { return roctx().on; }

void roctx_push(const std::string& name) {
  if (roctx().on) roctx().push(name.c_str());
}

void roctx_pop() {
  if (roctx().on) roctx().pop();
}

int mode() {
  State& s = st();
  int m = s.mode.load(std::memory_order_relaxed);
  if (m >= 0) return m;
  std::lock_guard<std::mutex> g(s.mu);
  if (s.mode.load() < 0) init_locked(s, std::getenv("ZEST_TRACE"));
  return s.mode.load();
}

void set_output(const std::string& path) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  init_locked(s, path.c_str());
}

uint64_t now_us() {
  return uint64_t(std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - st().t0).count());
}

void log(const char* cat, const std::string& msg) {
  if (mode() == kLog) {
    std::fprintf(stderr, "[zest +%.3fms %u] %s: %s\n", double(now_us()) / 1000.0, tid(), cat, msg.c_str());
    return;
  }
  if (mode() == kFile) {
    std::string e = "{\"ph\":\"i\",\"s\":\"t\",\"cat\":" + json::escape(cat) + ",\"name\":" + json::escape(msg) +
                    ",\"ts\":" + std::to_string(now_us()) + ",\"pid\":" + std::to_string(::getpid()) +
                    ",\"tid\":" + std::to_string(tid()) + "}";
    std::lock_guard<std::mutex> g(st().mu);
    st().events.push_back(std::move(e));
  }
}

void complete(const char* cat, const std::string& name, uint64_t ts, uint64_t dur, const std::string& args) {
  if (mode() == kLog) {
    std::fprintf(stderr, "[zest +%.3fms %u] %s: %s (%.3f ms)%s%s\n", double(ts) / 1000.0, tid(), cat, name.c_str(),
                 double(dur) / 1000.0, args.empty() ? "" : " ", args.c_str());
    return;
  }
  if (mode() != kFile) return;
  std::string e = "{\"ph\":\"X\",\"cat\":" + json::escape(cat) + ",\"name\":" + json::escape(name) +
                  ",\"ts\":" + std::to_string(ts) + ",\"dur\":" + std::to_string(dur) +
                  ",\"pid\":" + std::to_string(::getpid()) + ",\"tid\":" + std::to_string(tid());
  if (!args.empty()) e += ",\"args\":{" + args + "}";
  e += "}";
  std::lock_guard<std::mutex> g(st().mu);
  st().events.push_back(std::move(e));
}

void counter(const std::string& name, double value) {
  if (mode() != kFile) return;
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.6g", value);
  std::string e = "{\"ph\":\"C\",\"name\":" + json::escape(name) + ",\"ts\":" + std::to_string(now_us()) +
                  ",\"pid\":" + std::to_string(::getpid()) + ",\"args\":{\"value\":" + buf + "}}";
  std::lock_guard<std::mutex> g(st().mu);
  st().events.push_back(std::move(e));
}

void flush() {
  State& s = st();
  if (s.mode.load() != kFile) return;
  std::lock_guard<std::mutex> g(s.mu);
  std::FILE* f = std::fopen(s.path.c_str(), "w");
  if (!f) return;
  std::fputs("{\"traceEvents\":[\n", f);
  for (size_t i = 0; i < s.events.size(); ++i) {
    std::fputs(s.events[i].c_str(), f);
    std::fputs(i + 1 < s.events.size() ? ",\n" : "\n", f);
  }
  std::fputs("],\"displayTimeUnit\":\"ms\"}\n", f);
  std::fclose(f);
}

}  // namespace zest::trace
