// HBM that the ranks of one node can map from each other without hipIpcOpenMemHandle.
//
// The arena is one reserved virtual range backed by `chunk`-sized physical allocations
// (hipMemCreate, exportable as POSIX file descriptors = dmabufs).  A peer receives the fds over a
// Unix socket (SCM_RIGHTS, zest_amd/engine.py::map_peer_arenas), imports each with
// hipMemImportFromShareableHandle and maps them contiguously into its own reserved range, with
// read/write access for its own device (over xGMI when the memory lives on another GPU).
//
// Why: importing a >= 2 GiB torch allocation with hipIpcOpenMemHandle hung on the MI355X box (two
// ranks on one GPU; 64 and 512 MiB imports took < 2 ms), while a 16 GiB VMM arena of 32 x 512 MiB or
// 8 x 2 GiB chunks imported and mapped in 22-43 ms with the data intact
// (tools/experiments/vmm_ipc_probe.cpp; profiles/ipc_import_sizes_r3.txt, vmm_ipc_probe_r3.txt).
//
// Torch sees a mapping through DLPack (kDLROCM): the capsule's deleter holds a reference, so the
// mapping outlives every tensor view of it.
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <signal.h>
#include <pybind11/stl.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

void vcheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

hipMemAllocationProp device_prop(int device) {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

size_t granularity(int device) {
  const hipMemAllocationProp p = device_prop(device);
  size_t g = 0;
  vcheck(hipMemGetAllocationGranularity(&g, &p, hipMemAllocationGranularityRecommended), "granularity");
  return g ? g : 4096;
}

// Bytes of live mappings in this process, own and imported (vmm_live(): leak diagnostics).
std::atomic<int64_t> g_live_own{0}, g_live_imported{0};

// One contiguous virtual range mapped onto n physical chunks (own or imported).
struct VmmMapping {
  uint8_t* va = nullptr;
  size_t chunk = 0, size = 0;
  int device = 0;  // device that accesses it (owner's device, or the importer's)
  bool imported = false;
  bool counted = false;
  std::vector<hipMemGenericAllocationHandle_t> h;

  ~VmmMapping() {
    if (counted) (imported ? g_live_imported : g_live_own) -= int64_t(size);
    if (!va) return;
    (void)hipDeviceSynchronize();  // no kernel or copy may still touch the range
    for (size_t k = 0; k < h.size(); ++k) {
      (void)hipMemUnmap(va + k * chunk, chunk);
      (void)hipMemRelease(h[k]);
    }
    (void)hipMemAddressFree(va, size);
  }

  void reserve(size_t n_chunks) {
    size = n_chunks * chunk;
    void* p = nullptr;
    vcheck(hipMemAddressReserve(&p, size, 0, nullptr, 0), "hipMemAddressReserve");
    va = static_cast<uint8_t*>(p);
  }
  void grant() {
    if (!counted) {
      (imported ? g_live_imported : g_live_own) += int64_t(size);
      counted = true;
    }
    hipMemAccessDesc acc{};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = device;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    vcheck(hipMemSetAccess(va, size, &acc, 1), "hipMemSetAccess");
  }
};

std::shared_ptr<VmmMapping> vmm_alloc(size_t nbytes, int device, size_t chunk) {
  vcheck(hipSetDevice(device), "hipSetDevice");
  const size_t g = granularity(device);
  chunk = (std::max<size_t>(chunk, g) + g - 1) / g * g;
  auto m = std::make_shared<VmmMapping>();
  m->chunk = chunk;
  m->device = device;
  const size_t n = (std::max<size_t>(nbytes, 1) + chunk - 1) / chunk;
  m->reserve(n);
  const hipMemAllocationProp prop = device_prop(device);
  for (size_t k = 0; k < n; ++k) {
    hipMemGenericAllocationHandle_t h;
    vcheck(hipMemCreate(&h, chunk, &prop, 0), "hipMemCreate");
    m->h.push_back(h);
    vcheck(hipMemMap(m->va + k * chunk, chunk, 0, h, 0), "hipMemMap");
  }
  m->grant();
  return m;
}

// Fresh fds for every chunk (the caller sends and then closes them).
std::vector<int> vmm_export(const VmmMapping& m) {
  if (m.imported) throw std::runtime_error("only the owner exports its chunks");
  std::vector<int> fds;
  for (auto h : m.h) {
    int fd = -1;
    vcheck(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0), "export");
    fds.push_back(fd);
  }
  return fds;
}

// Map a peer's chunks (fds received from it; not closed here) for `device`.
std::shared_ptr<VmmMapping> vmm_import(const std::vector<int>& fds, size_t chunk, int device) {
  vcheck(hipSetDevice(device), "hipSetDevice");
  auto m = std::make_shared<VmmMapping>();
  m->chunk = chunk;
  m->device = device;
  m->imported = true;
  m->reserve(fds.size());
  // The HIP 7.0 runtime that PyTorch bundles reads the fd THROUGH `osHandle` (mov (%rsi),%edi before
  // hsa_amd_vmem_import_shareable_handle); ROCm 7.2's takes the fd as the pointer's value, like CUDA.
  int ver = 0;
  vcheck(hipRuntimeGetVersion(&ver), "hipRuntimeGetVersion");
  const bool by_pointer = ver < 70100000;
  for (size_t k = 0; k < fds.size(); ++k) {
    hipMemGenericAllocationHandle_t h;
    int fd = fds[k];
    void* os_handle = by_pointer ? static_cast<void*>(&fd) : reinterpret_cast<void*>(static_cast<intptr_t>(fd));
    vcheck(hipMemImportFromShareableHandle(&h, os_handle, hipMemHandleTypePosixFileDescriptor),
           "hipMemImportFromShareableHandle");
    m->h.push_back(h);
    vcheck(hipMemMap(m->va + k * chunk, chunk, 0, h, 0), "hipMemMap");
  }
  m->grant();
  return m;
}

// --- DLPack (v0.8 C ABI) ---------------------------------------------------------------------
struct DLDevice {
  int32_t device_type;  // kDLROCM = 10
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;  // kDLUInt = 1
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor* self);
};

struct DlCtx {
  std::shared_ptr<VmmMapping> keep;
  int64_t shape[1];
  int64_t strides[1];
  DLManagedTensor t;
};

void dl_delete(DLManagedTensor* self) { delete static_cast<DlCtx*>(self->manager_ctx); }

py::capsule vmm_dlpack(const std::shared_ptr<VmmMapping>& m, size_t nbytes) {
  if (nbytes > m->size) throw std::runtime_error("dlpack view larger than the mapping");
  auto* c = new DlCtx;
  c->keep = m;
  c->shape[0] = int64_t(nbytes);
  c->strides[0] = 1;
  c->t.dl_tensor = DLTensor{m->va, DLDevice{10, m->device}, 1, DLDataType{1, 8, 1}, c->shape, c->strides, 0};
  c->t.manager_ctx = c;
  c->t.deleter = dl_delete;
  return py::capsule(&c->t, "dltensor", [](PyObject* cap) {
    // an unconsumed capsule still owns the tensor; a consumer renamed it to "used_dltensor"
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (t && t->deleter) t->deleter(t);
    }
  });
}

void on_fatal(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

void bind_hip_vmm(py::module_& m) {
  // Diagnostics: print the native stack on SIGSEGV / SIGABRT (install before faulthandler.enable(),
  // which chains to it after the Python stack).
  m.def("install_fatal_backtrace", [] {
    signal(SIGSEGV, on_fatal);
    signal(SIGABRT, on_fatal);
  });
  py::class_<VmmMapping, std::shared_ptr<VmmMapping>>(m, "VmmMapping")
      .def_property_readonly("ptr", [](const VmmMapping& v) { return reinterpret_cast<uintptr_t>(v.va); })
      .def_readonly("size", &VmmMapping::size)
      .def_readonly("chunk", &VmmMapping::chunk)
      .def_readonly("device", &VmmMapping::device)
      .def_readonly("imported", &VmmMapping::imported)
      .def_property_readonly("n_chunks", [](const VmmMapping& v) { return v.h.size(); })
      .def("export_fds", [](const VmmMapping& v) {
        py::gil_scoped_release nogil;
        return vmm_export(v);
      })
      .def("dlpack", &vmm_dlpack, py::arg("nbytes"));
  m.def("vmm_granularity", &granularity, py::arg("device"));
  m.def("vmm_live", [] { return py::make_tuple(g_live_own.load(), g_live_imported.load()); },
        "bytes of live (own, imported) VMM mappings in this process");
  m.def("runtime_version", [] {
    int v = 0;
    vcheck(hipRuntimeGetVersion(&v), "hipRuntimeGetVersion");
    return v;
  });
  m.def(
      "vmm_alloc",
      [](size_t nbytes, int device, size_t chunk) {
        py::gil_scoped_release nogil;
        return vmm_alloc(nbytes, device, chunk);
      },
      py::arg("nbytes"), py::arg("device"), py::arg("chunk") = size_t(512) << 20);
  m.def(
      "vmm_import",
      [](const std::vector<int>& fds, size_t chunk, int device) {
        py::gil_scoped_release nogil;
        return vmm_import(fds, chunk, device);
      },
      py::arg("fds"), py::arg("chunk"), py::arg("device"));
}
