// Ready flags shared by the ranks of one node, for the peer-mapped exchanges (ipc / xgmi).
//
// A peer may read round k of an owner's arena only once the owner's kernels for round k finished.
// The first version made every rank's HOST wait for its own round k (event synchronize) and then
// meet the others in a host barrier before queueing the copies: per round, the issuing thread
// stalled on the GPU and on the slowest rank.  Here the wait moves onto the
// GPU: every rank owns one 32-bit counter in a small shared-memory page (one cache line per rank)
// that all ranks map and register with HIP.
//
//   owner:  after round k's kernels, a host function queued on a signal stream (behind an event
//           of the round's lane) stores seq_k into the owner's counter.  The host function runs
//           after the runtime saw the round complete, so its writes are visible system-wide
//           (the same guarantee the event synchronize gave).
//   reader: hipStreamWaitValue32(counter[owner] >= seq_k) on the exchange stream, then the
//           copies / the K8 gather.  The issuing thread never blocks.
//
// seq numbers grow monotonically for the lifetime of the mapping (identical on every rank: every
// rank signals every round, in the same order), so a wait can never be satisfied by an older step.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

constexpr size_t kSlotBytes = 64;  // one counter per cache line

void scheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct PeerSignals {
  int n = 0;
  size_t bytes = 0;
  uint8_t* host = nullptr;
  uint8_t* dev = nullptr;  // device address of the same pages
  bool registered = false;

  ~PeerSignals() {
    if (!host) return;
    if (registered) {
      // No wait command may still poll the page when it is unmapped, so the device is synchronized
      // -- after every slot is opened (0xFFFFFFFF), so that a wait on a rank that will never signal
      // again (it died, or this pull failed) cannot hang the teardown.  Safe for the other
      // ranks: a page is dropped only after a pull ended on every rank (the end of a pull is a
      // collective) or after a failure, and the next pull agrees on a fresh page.
      release();
      (void)hipDeviceSynchronize();
      (void)hipHostUnregister(host);
    }
    munmap(host, bytes);
  }
  void release() {
    for (int i = 0; i < n; ++i) __atomic_store_n(slot(i), 0xFFFFFFFFu, __ATOMIC_RELEASE);
  }
  uint32_t* slot(int i) const {
    if (i < 0 || i >= n) throw std::out_of_range("signal slot");
    return reinterpret_cast<uint32_t*>(host + size_t(i) * kSlotBytes);
  }
  void* dev_slot(int i) const {
    if (i < 0 || i >= n) throw std::out_of_range("signal slot");
    return dev + size_t(i) * kSlotBytes;
  }
};

// Map (and with `create`, make) the shared page at `path` for `n` ranks on `device`.
std::shared_ptr<PeerSignals> signals_open(const std::string& path, int n, bool create, int device) {
  if (n <= 0 || n > 1024) throw std::invalid_argument("signals_open: 1..1024 ranks");
  auto s = std::make_shared<PeerSignals>();
  s->n = n;
  s->bytes = (size_t(n) * kSlotBytes + 4095) / 4096 * 4096;
  const int fd = open(path.c_str(), O_RDWR | O_CLOEXEC | (create ? O_CREAT | O_EXCL : 0), 0600);
  if (fd < 0) throw std::runtime_error("signals_open " + path + ": " + std::strerror(errno));
  if (create && ftruncate(fd, off_t(s->bytes)) != 0) {
    const int e = errno;
    close(fd);
    throw std::runtime_error("signals_open ftruncate: " + std::string(std::strerror(e)));
  }
  struct stat st{};
  if (fstat(fd, &st) != 0 || size_t(st.st_size) < s->bytes) {
    close(fd);
    throw std::runtime_error("signals_open: " + path + " is smaller than " + std::to_string(s->bytes) + " bytes");
  }
  void* p = mmap(nullptr, s->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("signals_open mmap: " + std::string(std::strerror(errno)));
  s->host = static_cast<uint8_t*>(p);
  scheck(hipSetDevice(device), "hipSetDevice");
  scheck(hipHostRegister(s->host, s->bytes, hipHostRegisterMapped), "hipHostRegister (signals)");
  s->registered = true;
  void* d = nullptr;
  scheck(hipHostGetDevicePointer(&d, s->host, 0), "hipHostGetDevicePointer (signals)");
  s->dev = static_cast<uint8_t*>(d);
  return s;
}

struct SetCtx {
  uint32_t* slot;
  uint32_t value;
};

void set_slot(void* arg) {
  auto* c = static_cast<SetCtx*>(arg);
  __atomic_store_n(c->slot, c->value, __ATOMIC_RELEASE);
  delete c;
}

}  // namespace

void bind_hip_signals(py::module_& m) {
  py::class_<PeerSignals, std::shared_ptr<PeerSignals>>(m, "PeerSignals")
      .def_readonly("n", &PeerSignals::n)
      .def("value", [](const PeerSignals& s, int i) { return __atomic_load_n(s.slot(i), __ATOMIC_ACQUIRE); })
      .def("store", [](const PeerSignals& s, int i, uint32_t v) { __atomic_store_n(s.slot(i), v, __ATOMIC_RELEASE); })
      // Open every slot: no wait on this page blocks any more (a lost rank, a failed pull).
      .def("release", [](PeerSignals& s) { s.release(); })
      // Queue on `stream`: store `value` into slot i once everything queued before it has completed.
      .def("set_after",
           [](const PeerSignals& s, int i, uint32_t v, uintptr_t stream) {
             auto* c = new SetCtx{s.slot(i), v};
             const hipError_t e = hipLaunchHostFunc(reinterpret_cast<hipStream_t>(stream), set_slot, c);
             if (e != hipSuccess) {
               delete c;
               scheck(e, "hipLaunchHostFunc (signal)");
             }
           })
      // Queue on `stream`: nothing queued after this runs until slot i >= value.
      .def("wait_on",
           [](const PeerSignals& s, int i, uint32_t v, uintptr_t stream) {
             scheck(hipStreamWaitValue32(reinterpret_cast<hipStream_t>(stream), s.dev_slot(i), v, hipStreamWaitValueGte,
                                         0xFFFFFFFFu),
                    "hipStreamWaitValue32 (signal)");
           });
  m.def(
      "signals_open",
      [](const std::string& path, int n, bool create, int device) {
        py::gil_scoped_release nogil;
        return signals_open(path, n, create, device);
      },
      py::arg("path"), py::arg("n"), py::arg("create"), py::arg("device"));
  m.def("can_stream_wait_value", [](int device) {
    int v = 0;
    scheck(hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, device), "hipDeviceGetAttribute");
    return v != 0;
  });
}
