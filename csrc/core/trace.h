// Host tracing: Chrome-trace spans + debug log lines, switched by ZEST_TRACE.
//
//   ZEST_TRACE unset / "0"     tracing off (one relaxed atomic load per probe)
//   ZEST_TRACE=1               log lines "[zest +12.345ms tid] cat: msg" on stderr
//   ZEST_TRACE=/path/out.json  Chrome trace-event JSON written at exit (and on trace::flush())
//
//   ZEST_ROCTX=1               every span is also a roctx range (rocprofv3 --marker-trace shows
//                              fetch / verify / serve phases next to the kernels); the ROCm roctx
//                              library is dlopen'ed on first use, so the core has no link dependency
//
// The reference has no tracing; this is the host half of the design there.  The
// Python layer adds device spans (HIP event timings) to the same file via _core.trace_*.
#pragma once

#include <chrono>
#include <cstdint>
#include <sstream>
#include <string>

namespace zest::trace {

enum Mode : int { kOff = 0, kLog = 1, kFile = 2 };
int mode();  // cached from the environment on first use
inline bool enabled() { return mode() != kOff; }

uint64_t now_us();
void log(const char* cat, const std::string& msg);
// Complete event ("ph":"X").
void complete(const char* cat, const std::string& name, uint64_t ts_us, uint64_t dur_us, const std::string& args_json = "");
void counter(const std::string& name, double value);
void flush();
void set_output(const std::string& path);  // override ZEST_TRACE at runtime (tests)
bool roctx_enabled();                      // ZEST_ROCTX=1 and the roctx library loaded
void roctx_push(const std::string& name);
void roctx_pop();

class Span {
 public:
  Span(const char* cat, std::string name) : cat_(cat), on_(enabled()), rx_(roctx_enabled()) {
    if (on_ || rx_) name_ = std::move(name);
    if (on_) t0_ = now_us();
    if (rx_) roctx_push(std::string(cat_) + ": " + name_);
  }
  ~Span() {
    if (rx_) roctx_pop();
    if (on_) complete(cat_, name_, t0_, now_us() - t0_, args_);
  }
  void arg(const std::string& json_kv) {  // e.g. "\"bytes\":123"
    if (on_) args_ += (args_.empty() ? "" : ",") + json_kv;
  }

 private:
  const char* cat_;
  bool on_, rx_;
  std::string name_, args_;
  uint64_t t0_ = 0;
};

}  // namespace zest::trace

#define ZTRACE(cat, expr)                             \
  do {                                                \
    if (::zest::trace::enabled()) {                   \
      std::ostringstream _zt_os;                      \
      _zt_os << expr;                                 \
      ::zest::trace::log(cat, _zt_os.str());          \
    }                                                 \
  } while (0)
