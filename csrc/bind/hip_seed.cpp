// HBM seeding: a BEP XET server whose piece provider reads serialized xorbs resident in GPU
// memory (BASELINE config "Mixtral-8x7B seed mode: serve xorbs from 288 GB HBM").
//
// Each request [range_start, range_end) of a registered xorb is copied HBM -> a per-connection
// pinned staging buffer (hipMemcpyAsync on a per-thread stream) and written to the socket straight
// from that buffer (zero-copy CacheHit), so a served byte crosses PCIe once and is never copied on
// the host.  Xorbs not in HBM fall through to the disk cache like `zest serve`.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "bt_server.h"
#include "config.h"
#include "storage.h"
#include "xet_hash.h"

namespace py = pybind11;
using namespace zest;

namespace {

struct XorbLoc {
  uint64_t dev_off;                 // serialized run start inside the device arena
  std::vector<uint64_t> ends;       // serialized end offset of each chunk (relative to dev_off)
  uint32_t first = 0;               // xorb chunk index of the run's first chunk (partial runs)
};

// Per connection thread: pinned staging for one response, the stream its D2H copies run on, and one
// event per piece.  A thread serves one request at a time, so the next response reuses them only after
// the previous one was sent.
struct Staging {
  uint8_t* host = nullptr;
  size_t cap = 0;
  hipStream_t stream = nullptr;
  std::vector<hipEvent_t> ev;
  ~Staging() {
    if (stream) (void)hipStreamSynchronize(stream);
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    if (host) (void)hipHostFree(host);
    if (stream) (void)hipStreamDestroy(stream);
  }
  void ensure(size_t n, size_t pieces) {
    while (ev.size() < pieces) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) throw Error("HipError", "hipEventCreate");
      ev.push_back(e);
    }
    if (n <= cap) return;
    if (host) (void)hipHostFree(host);
    host = nullptr;
    cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&host), n, hipHostMallocDefault) != hipSuccess)
      throw Error("HipError", "hipHostMalloc staging");
    cap = n;
  }
};

class HbmSeeder {
 public:
  HbmSeeder(uintptr_t arena, uint64_t arena_bytes, int device, int port, bool disk_fallback)
      : arena_(reinterpret_cast<const uint8_t*>(arena)), arena_n_(arena_bytes), device_(device),
        cfg_(Config::from_env()) {
    if (disk_fallback) {
      registry_.scan(cfg_);
      cache_ = std::make_unique<storage::XorbCache>(cfg_, &registry_);
    }
    server_ = std::make_unique<bt::BtServer>(
        cfg_, cache_.get(),
        [this](const std::array<uint8_t, 32>&, const std::string& hex, uint32_t a, uint32_t b) {
          return provide(hex, a, b);
        },
        port);
  }
  ~HbmSeeder() { stop(); }

  void add_xorb(const std::string& hex, uint64_t dev_off, std::vector<uint64_t> ends, uint32_t first) {
    if (ends.empty() || dev_off + ends.back() > arena_n_) throw Error("InvalidRange", "xorb outside arena");
    std::unique_lock<std::shared_mutex> g(mu_);
    index_[hex].push_back(XorbLoc{dev_off, std::move(ends), first});  // several runs per xorb allowed
  }
  size_t count() const {
    std::shared_lock<std::shared_mutex> g(mu_);
    return index_.size();
  }
  void start() { server_->start(); }
  void stop() {
    if (server_) server_->stop();
  }
  uint16_t port() const { return server_->port(); }
  bt::ServerStats stats() const { return server_->stats(); }

 private:
  std::optional<storage::CacheHit> provide(const std::string& hex, uint32_t a, uint32_t b) {
    uint64_t lo, hi;
    {
      std::shared_lock<std::shared_mutex> g(mu_);
      auto it = index_.find(hex);
      if (it == index_.end()) return std::nullopt;
      const XorbLoc* hit = nullptr;
      uint32_t bb = b;
      for (const XorbLoc& x : it->second) {  // first run covering [a, b)
        const uint32_t n = x.first + uint32_t(x.ends.size());
        const uint32_t want_end = b == 0 ? n : b;
        if (a >= x.first && a < want_end && want_end <= n) {
          hit = &x;
          bb = want_end;
          break;
        }
      }
      if (!hit) return std::nullopt;
      const uint32_t ra = a - hit->first, rb = bb - hit->first;
      lo = hit->dev_off + (ra ? hit->ends[ra - 1] : 0);
      hi = hit->dev_off + hit->ends[rb - 1];
    }
    thread_local std::shared_ptr<Staging> st;
    if (!st) {
      st = std::make_shared<Staging>();
      (void)hipSetDevice(device_);
      if (hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking) != hipSuccess)
        throw Error("HipError", "hipStreamCreate");
    }
    // The response is copied HBM -> pinned in pieces of kPiece (ZEST_SEED_PIECE_MB, default 8)
    // queued back to back, each followed by an event: the server sends piece k while piece k + 1 is
    // still in flight (ready() waits for the piece a slice needs), instead of copying the whole
    // run (up to 64 MiB) and synchronizing before the first byte goes out.
    static const size_t kPiece = [] {
      const char* v = std::getenv("ZEST_SEED_PIECE_MB");
      const size_t mb = v && *v ? size_t(std::strtoull(v, nullptr, 10)) : 8;
      return std::max<size_t>(1, mb) << 20;
    }();
    const size_t len = size_t(hi - lo);
    const size_t pieces = std::max<size_t>(1, (len + kPiece - 1) / kPiece);
    st->ensure(len, pieces);
    for (size_t k = 0; k < pieces; ++k) {
      const size_t o = k * kPiece, n = std::min(kPiece, len - o);
      if ((n && hipMemcpyAsync(st->host + o, arena_ + lo + o, n, hipMemcpyDeviceToHost, st->stream) != hipSuccess) ||
          hipEventRecord(st->ev[k], st->stream) != hipSuccess)
        throw Error("HipError", "HBM -> host copy");
    }
    storage::CacheHit h;
    h.chunk_offset = a;
    h.ext = st->host;
    h.ext_len = len;
    h.keep = st;
    Staging* sp = st.get();
    h.ready = [sp](size_t upto) {
      if (!upto) return;
      const size_t k = (upto - 1) / kPiece;
      if (hipEventSynchronize(sp->ev[std::min(k, sp->ev.size() - 1)]) != hipSuccess)
        throw Error("HipError", "HBM -> host copy");
    };
    return h;
  }

  const uint8_t* arena_;
  uint64_t arena_n_;
  int device_;
  Config cfg_;
  storage::XorbRegistry registry_;
  std::unique_ptr<storage::XorbCache> cache_;
  std::unique_ptr<bt::BtServer> server_;
  mutable std::shared_mutex mu_;
  std::unordered_map<std::string, std::vector<XorbLoc>> index_;
};

}  // namespace

void bind_hip_seed(py::module_& m) {
  py::class_<HbmSeeder>(m, "HbmSeeder", "BEP XET seeder serving serialized xorbs from HBM")
      .def(py::init<uintptr_t, uint64_t, int, int, bool>(), py::arg("arena_ptr"), py::arg("arena_bytes"),
           py::arg("device") = 0, py::arg("port") = 0, py::arg("disk_fallback") = false)
      .def("add_xorb", &HbmSeeder::add_xorb, py::arg("xet_hex"), py::arg("dev_off"), py::arg("chunk_ends"),
           py::arg("first_chunk") = 0)
      .def("start", &HbmSeeder::start)
      .def("stop", [](HbmSeeder& s) {
        py::gil_scoped_release nogil;
        s.stop();
      })
      .def_property_readonly("port", &HbmSeeder::port)
      .def("__len__", &HbmSeeder::count)
      .def("stats", [](const HbmSeeder& s) {
        auto st = s.stats();
        py::dict d;
        d["active_peers"] = st.active_peers;
        d["total_peers"] = st.total_peers;
        d["chunks_served"] = st.chunks_served;
        d["chunk_units"] = st.chunk_units;
        d["bytes_served"] = st.bytes_served;
        d["not_found"] = st.not_found;
        d["rejected"] = st.rejected;
        d["lookup_s"] = double(st.lookup_ns) / 1e9;
        d["wait_s"] = double(st.wait_ns) / 1e9;
        d["send_s"] = double(st.send_ns) / 1e9;
        return d;
      });
}
