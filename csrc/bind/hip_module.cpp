// pybind11 bindings for the HIP/CDNA4 kernel library (`zest_amd._hip`).  All entry points take
// raw device pointers (ints) and a hipStream_t (int, e.g. torch.cuda.current_stream().cuda_stream);
// shape/bounds validation happens in zest_amd/ops before launch.
#include <hip/hip_runtime.h>

#include <cstring>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstddef>
#include <stdexcept>
#include <string>
#include <vector>

#include <map>
#include <mutex>
#include <utility>

#include "../gpu/zgpu.h"
#include "../gpurt/pinned.h"

namespace py = pybind11;

void bind_hip_seed(py::module_& m);  // hip_seed.cpp
void bind_hip_pull(py::module_& m);  // hip_pull.cpp
void bind_hip_vmm(py::module_& m);   // hip_vmm.cpp
void bind_hip_signals(py::module_& m);  // hip_signals.cpp

namespace {

// host_malloc'd buffers: address -> (mapped length, registered mapping?) for host_free
std::map<uintptr_t, std::pair<size_t, bool>>& host_allocs() {
  static std::map<uintptr_t, std::pair<size_t, bool>> m;
  return m;
}
std::mutex& host_allocs_mu() {
  static std::mutex mu;
  return mu;
}

template <typename T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

PYBIND11_MODULE(_hip, m) {
  m.doc() = "zest HIP kernels for AMD Instinct MI355X (gfx950)";
  m.attr("TERM_BYTES") = sizeof(ZgTerm);
  m.attr("CHUNK_BYTES") = sizeof(ZgChunk);
  m.attr("MERKLE_JOB_BYTES") = sizeof(ZgMerkleJob);
  m.attr("ARCH") = "gfx950";
  bind_hip_seed(m);
  bind_hip_pull(m);
  bind_hip_vmm(m);
  bind_hip_signals(m);

  m.def("device_count", &zg_device_count);
  // Pinned host memory (hipHostMalloc: exact size, unlike torch's power-of-two caching host
  // allocator) and raw async copies on a caller-provided stream.
  // Pinned host memory for origins / staging: anonymous THP mapping faulted in by several threads,
  // then hipHostRegister (gpurt/pinned.h; 72 vs 191 ms per GiB against hipHostMalloc on the box, and
  // the same H2D rate), falling back to hipHostMalloc.
  m.def("host_malloc", [](size_t n) {
    zest::gpurt::PinnedBuf b;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = b.alloc(n ? n : 1);
    }
    if (!ok) throw std::runtime_error("host_malloc: pinning " + std::to_string(n) + " bytes failed");
    const size_t len = b.size();
    const bool mapped = b.mapped();
    uint8_t* p = b.release();
    std::lock_guard<std::mutex> g(host_allocs_mu());
    host_allocs()[reinterpret_cast<uintptr_t>(p)] = {len, mapped};
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("host_free", [](uintptr_t p) {
    std::pair<size_t, bool> a{0, false};
    {
      std::lock_guard<std::mutex> g(host_allocs_mu());
      auto it = host_allocs().find(p);
      if (it == host_allocs().end()) throw std::invalid_argument("host_free: not from host_malloc");
      a = it->second;
      host_allocs().erase(it);
    }
    py::gil_scoped_release nogil;
    zest::gpurt::PinnedBuf::free_raw(reinterpret_cast<uint8_t*>(p), a.first, a.second);
  });
  // Let the current device's copy engines read `peer`'s memory directly over xGMI (IPC exchange).
  m.def("enable_peer_access", [](int peer) {
    int dev = 0;
    check(hipGetDevice(&dev), "hipGetDevice");
    if (peer == dev) return true;
    int can = 0;
    check(hipDeviceCanAccessPeer(&can, dev, peer), "hipDeviceCanAccessPeer");
    if (!can) return false;
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    else check(e, "hipDeviceEnablePeerAccess");
    return true;
  });
  // Raw HIP IPC (dmabuf) of a device allocation, without torch's IPC wrapper (which also exports
  // an event and a ref-counter file): export the allocation holding `ptr` as bytes, open a peer's.
  // Returns (handle bytes, offset of ptr from the start of its allocation).
  m.def("ipc_get_handle", [](uintptr_t ptr) {
    hipIpcMemHandle_t h;
    check(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)), "hipIpcGetMemHandle");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    check(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)), "hipMemGetAddressRange");
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof h),
                          uint64_t(ptr - reinterpret_cast<uintptr_t>(base)));
  });
  m.def("ipc_open_handle", [](const py::bytes& b) {
    const std::string s = b;
    if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("ipc handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof h);
    void* p = nullptr;
    {
      py::gil_scoped_release nogil;
      check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    }
    return reinterpret_cast<uintptr_t>(p);
  });
  m.def("ipc_close_handle", [](uintptr_t p) {
    check(hipIpcCloseMemHandle(reinterpret_cast<void*>(p)), "hipIpcCloseMemHandle");
  });
  m.def("memcpy_async", [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t st) {
    check(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n, hipMemcpyDefault, S(st)),
          "hipMemcpyAsync");
  });
  // Stream-order `st` after a raw hipEvent_t (DeviceXetPull.wait_item's item events).
  m.def("stream_wait_event", [](uintptr_t st, uintptr_t ev) {
    check(hipStreamWaitEvent(S(st), reinterpret_cast<hipEvent_t>(ev), 0), "hipStreamWaitEvent");
  });
  // K8 (xgmi exchange): one launch pulls every (peer src, local dst, bytes) segment.
  m.def("peer_gather", [](const std::vector<uint64_t>& src, const std::vector<uint64_t>& dst,
                          const std::vector<uint64_t>& n, uintptr_t st) {
    if (src.size() != dst.size() || src.size() != n.size() || src.size() > size_t(kZgMaxPeerSegs))
      throw std::invalid_argument("peer_gather: need equal-length src/dst/n lists of at most 16 segments");
    ZgPeerSegs s{};
    s.nseg = int(src.size());
    for (size_t i = 0; i < src.size(); ++i) {
      if ((src[i] & 15) != (dst[i] & 15)) throw std::invalid_argument("peer_gather: src/dst not congruent mod 16");
      s.src[i] = src[i];
      s.dst[i] = dst[i];
      s.n[i] = n[i];
    }
    check(zg_peer_gather(&s, S(st)), "zg_peer_gather");
  });
  m.def("index_terms", [](uintptr_t src, uintptr_t terms, int n, uintptr_t chunks, uintptr_t err, uintptr_t st) {
    check(zg_index_terms(P<const uint8_t>(src), P<const ZgTerm>(terms), n, P<ZgChunk>(chunks),
                         P<unsigned long long>(err), S(st)),
          "zg_index_terms");
  });
  m.def("index_scratch_bytes", &zg_index_scratch_bytes);
  m.def("index_terms_scan", [](uintptr_t src, uint64_t src_n, uintptr_t terms, int n, uintptr_t chunks, uintptr_t err,
                               uintptr_t scratch, size_t scratch_bytes, uintptr_t st) {
    check(zg_index_terms_scan(P<const uint8_t>(src), src_n, P<const ZgTerm>(terms), n, P<ZgChunk>(chunks),
                              P<unsigned long long>(err), P<uint8_t>(scratch), scratch_bytes, S(st)),
          "zg_index_terms_scan");
  });
  m.def("place_chunks", [](uintptr_t src, uint64_t src_n, uintptr_t dst, uint64_t dst_n, uintptr_t chunks, int n,
                           uint64_t lo, uint64_t hi, uintptr_t err, uintptr_t st, uintptr_t clip_scratch) {
    check(zg_place_chunks(P<const uint8_t>(src), src_n, P<uint8_t>(dst), dst_n, P<const ZgChunk>(chunks), n, lo, hi,
                          P<uint8_t>(clip_scratch), P<unsigned long long>(err), S(st)),
          "zg_place_chunks");
  }, py::arg("src"), py::arg("src_n"), py::arg("dst"), py::arg("dst_n"), py::arg("chunks"), py::arg("n"),
     py::arg("lo"), py::arg("hi"), py::arg("err"), py::arg("stream"), py::arg("clip_scratch") = 0);
  m.attr("CLIP_SCRATCH_BYTES") = ZG_CLIP_SCRATCH_BYTES;
  m.def("hash_scratch_bytes", [](int n, uint64_t total_bytes) { return zg_hash_scratch_bytes(n, total_bytes); });
  m.def("ingest_scratch_bytes", [](int n, uint64_t total_bytes) { return zg_ingest_scratch_bytes(n, total_bytes); });
  m.def("hash_chunks", [](uintptr_t dst, uint64_t dst_n, uintptr_t chunks, int n, uintptr_t hashes, uintptr_t sizes,
                          uint32_t base, uintptr_t st, uintptr_t scratch, size_t scratch_bytes) {
    check(zg_hash_chunks(P<const uint8_t>(dst), dst_n, P<const ZgChunk>(chunks), n, P<uint8_t>(hashes),
                         P<uint64_t>(sizes), base, P<uint8_t>(scratch), scratch_bytes, S(st)),
          "zg_hash_chunks");
  }, py::arg("dst"), py::arg("dst_n"), py::arg("chunks"), py::arg("n"), py::arg("hashes"), py::arg("sizes"),
     py::arg("base"), py::arg("stream"), py::arg("scratch") = 0, py::arg("scratch_bytes") = 0);
  m.def("ingest_chunks", [](uintptr_t src, uint64_t src_n, uintptr_t dst, uint64_t dst_n, uintptr_t chunks, int n,
                            bool has_compressed, uintptr_t err, uintptr_t hashes, uintptr_t sizes, uint32_t base,
                            uintptr_t st, uintptr_t scratch, size_t scratch_bytes) {
    check(zg_ingest_chunks(P<const uint8_t>(src), src_n, P<uint8_t>(dst), dst_n, P<const ZgChunk>(chunks), n,
                           has_compressed ? 1 : 0, P<unsigned long long>(err), P<uint8_t>(hashes), P<uint64_t>(sizes),
                           base, P<uint8_t>(scratch), scratch_bytes, S(st)),
          "zg_ingest_chunks");
  }, py::arg("src"), py::arg("src_n"), py::arg("dst"), py::arg("dst_n"), py::arg("chunks"), py::arg("n"),
     py::arg("has_compressed"), py::arg("err"), py::arg("hashes"), py::arg("sizes"), py::arg("base"), py::arg("stream"),
     py::arg("scratch"), py::arg("scratch_bytes"),
     "fused ingest: LZ4/BG4 decode of compressed chunks, then one pass that places raw chunks and hashes all");
  m.def("lz4_decode", [](uintptr_t src, uint64_t src_n, uintptr_t dst, uint64_t dst_n, uintptr_t chunks, int n,
                         uintptr_t err, uintptr_t st, int grid_cap, uintptr_t rec_scratch, size_t rec_scratch_bytes,
                         bool pair) {
    if (pair)
      check(zg_lz4_pair_decode(P<const uint8_t>(src), src_n, P<uint8_t>(dst), dst_n, P<const ZgChunk>(chunks), n,
                               P<unsigned long long>(err), grid_cap, S(st)),
            "zg_lz4_pair_decode");
    else if (rec_scratch)
      check(zg_lz4_decode_records(P<const uint8_t>(src), src_n, P<uint8_t>(dst), dst_n, P<const ZgChunk>(chunks), n,
                                  P<unsigned long long>(err), P<uint8_t>(rec_scratch), rec_scratch_bytes, S(st)),
            "zg_lz4_decode_records");
    else
      check(zg_lz4_batched_decode_grid(P<const uint8_t>(src), src_n, P<uint8_t>(dst), dst_n, P<const ZgChunk>(chunks),
                                       n, P<unsigned long long>(err), grid_cap, S(st)),
            "zg_lz4_batched_decode");
  }, py::arg("src"), py::arg("src_n"), py::arg("dst"), py::arg("dst_n"), py::arg("chunks"), py::arg("n"),
     py::arg("err"), py::arg("stream"), py::arg("grid_cap") = 0, py::arg("rec_scratch") = 0,
     py::arg("rec_scratch_bytes") = 0, py::arg("pair") = false,
     "K3 alone on the compressed chunks of `chunks` (raw ones are skipped): `pair` = producer/consumer wave "
     "pairs (grid_cap in pairs), else the two-kernel records decoder with rec_scratch (>= "
     "lz4_rec_scratch_bytes), else the one-kernel batched decoder");
  m.def("lz4_rec_scratch_bytes", [](int n, uint64_t src_n) { return zg_lz4_rec_scratch_bytes(n, src_n); });
  m.def("hash_ranges", [](uintptr_t buf, uintptr_t offs, uintptr_t lens, int n, uintptr_t out, int key_mode,
                          uintptr_t st, uintptr_t scratch, size_t scratch_bytes) {
    check(zg_hash_ranges(P<const uint8_t>(buf), P<const uint64_t>(offs), P<const uint32_t>(lens), n,
                         P<uint8_t>(out), key_mode, P<uint8_t>(scratch), scratch_bytes, S(st)),
          "zg_hash_ranges");
  }, py::arg("buf"), py::arg("offs"), py::arg("lens"), py::arg("n"), py::arg("out"), py::arg("key_mode"),
     py::arg("stream"), py::arg("scratch") = 0, py::arg("scratch_bytes") = 0);
  m.def("compress_chunks", [](uintptr_t data, uintptr_t offs, uintptr_t lens, int n, int bg4, uintptr_t scratch,
                              uint64_t in_slot, uintptr_t out, uint64_t out_slot, uintptr_t out_len, uint32_t hc64,
                              uint32_t hc256, uintptr_t st) {
    check(zg_compress_chunks(P<const uint8_t>(data), P<const uint64_t>(offs), P<const uint32_t>(lens), n, bg4,
                             P<uint8_t>(scratch), in_slot, P<uint8_t>(out), out_slot, P<uint32_t>(out_len), hc64, hc256,
                             S(st)),
          "zg_compress_chunks");
  });
  m.def("pack_frames", [](uintptr_t src, uintptr_t clen, uintptr_t ulen, uintptr_t scheme, uintptr_t out_off, int n,
                          uintptr_t out, uintptr_t st) {
    check(zg_pack_frames(P<const uint64_t>(src), P<const uint32_t>(clen), P<const uint32_t>(ulen),
                         P<const uint8_t>(scheme), P<const uint64_t>(out_off), n, P<uint8_t>(out), S(st)),
          "zg_pack_frames");
  });
  m.def("merkle_scratch_bytes", &zg_merkle_scratch_bytes);
  m.def("merkle", [](uintptr_t hashes, uintptr_t sizes, uintptr_t jobs, int n_jobs, uintptr_t roots,
                     uintptr_t scratch, uint64_t scratch_bytes, uintptr_t st) {
    check(zg_merkle(P<const uint8_t>(hashes), P<const uint64_t>(sizes), P<const ZgMerkleJob>(jobs), n_jobs,
                    P<uint8_t>(roots), P<uint8_t>(scratch), scratch_bytes, S(st)),
          "zg_merkle");
  });
  m.def("compare_hashes", [](uintptr_t got, uintptr_t want, int n, uintptr_t err, uintptr_t st) {
    check(zg_compare_hashes(P<const uint8_t>(got), P<const uint8_t>(want), n, P<unsigned long long>(err), S(st)),
          "zg_compare_hashes");
  });
  m.def("cdc_candidates", [](uintptr_t data, uint64_t n, uint64_t mask, uintptr_t out, uintptr_t count, uint64_t cap,
                             uintptr_t st) {
    check(zg_cdc_candidates(P<const uint8_t>(data), n, mask, P<uint64_t>(out), P<unsigned long long>(count), cap,
                            S(st)),
          "zg_cdc_candidates");
  });
  m.def("fill_synthetic", [](uintptr_t dst, uint64_t n, uint64_t seed, uint64_t off, int mode, uintptr_t st) {
    check(zg_fill_synthetic(P<uint8_t>(dst), n, seed, off, mode, S(st)), "zg_fill_synthetic");
  });
  m.def("sha1_info_hash", [](uintptr_t hashes, int n, uintptr_t out, uintptr_t st) {
    check(zg_sha1_info_hash(P<const uint8_t>(hashes), n, P<uint8_t>(out), S(st)), "zg_sha1_info_hash");
  });
  m.def("pack_chunks", [](uintptr_t data, uintptr_t data_off, uintptr_t lens, uintptr_t out_off, int n, uintptr_t out,
                          uintptr_t st) {
    check(zg_pack_chunks(P<const uint8_t>(data), P<const uint64_t>(data_off), P<const uint32_t>(lens),
                         P<const uint64_t>(out_off), n, P<uint8_t>(out), S(st)),
          "zg_pack_chunks");
  });
}
