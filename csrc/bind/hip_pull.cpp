// pybind11 face of the native device-direct pull (csrc/gpurt/device_pull.{h,cpp}): fetch a Xet
// file's terms through the cache -> P2P -> CDN waterfall into pinned staging and decode + BLAKE3 +
// Merkle-verify them on the GPU into caller-provided HBM.  North-star path for
// `zest_amd.pull(..., device=...)` and the owner fetch of `parallel.swarm_pull`.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../gpurt/device_pull.h"
#include "term_py.h"

namespace py = pybind11;
using zest::gpurt::DeviceXetPull;
using zest::gpurt::DevicePullOptions;
using zest::gpurt::PullRequest;

namespace {

py::list pull_files_py(DeviceXetPull& self, const std::vector<std::tuple<std::string, uintptr_t, uint64_t>>& files) {
  std::vector<PullRequest> req;
  for (const auto& f : files) req.push_back({std::get<0>(f), std::get<1>(f), std::get<2>(f)});
  std::vector<zest::gpurt::PullFileStats> st;
  {
    py::gil_scoped_release nogil;  // the fetch may talk to a hub served from this process
    st = self.pull_files(req);
  }
  py::list out;
  for (auto& s : st) {
    py::dict d;
    d["bytes"] = s.bytes;
    d["terms"] = s.terms;
    d["chunks"] = s.chunks;
    d["seconds"] = s.seconds;
    d["fetched_bytes"] = s.fetched_bytes;
    d["chunk_lens"] = py::bytes(reinterpret_cast<const char*>(s.chunk_lens.data()), 4 * s.chunk_lens.size());
    out.append(d);
  }
  return out;
}

}  // namespace

void bind_hip_pull(py::module_& m) {
  py::class_<DeviceXetPull>(m, "DeviceXetPull", "Xet pull with GPU ingest + verification into HBM")
      .def(py::init([](const std::string& repo, const std::string& revision, const std::string& repo_type, bool p2p,
                       std::vector<std::string> peers, std::optional<std::string> tracker, bool dht,
                       std::vector<std::string> boot, int device, size_t staging, int threads) {
             DevicePullOptions o;
             o.repo = repo;
             o.revision = revision;
             o.repo_type = repo_type;
             o.p2p = p2p;
             o.peers = std::move(peers);
             o.tracker = std::move(tracker);
             o.dht = dht;
             o.dht_bootstrap = std::move(boot);
             o.device = device;
             o.staging_bytes = staging;
             o.threads = threads;
             // Authentication talks HTTP: release the GIL (the hub may be served from this process).
             py::gil_scoped_release nogil;
             return new DeviceXetPull(o);
           }),
           py::arg("repo"), py::arg("revision") = "main", py::arg("repo_type") = "model", py::arg("p2p") = true,
           py::arg("peers") = std::vector<std::string>{}, py::arg("tracker") = std::nullopt, py::arg("dht") = true,
           py::arg("dht_bootstrap") = std::vector<std::string>{}, py::arg("device") = 0,
           py::arg("staging_bytes") = size_t(1) << 30, py::arg("threads") = 16)
      .def("pull_file",
           [](DeviceXetPull& self, const std::string& hex, uintptr_t dst, uint64_t size) {
             return pull_files_py(self, {std::make_tuple(hex, dst, size)})[0].cast<py::dict>();
           },
           py::arg("xet_hash"), py::arg("dst_ptr"), py::arg("dst_size"))
      .def("pull_files", &pull_files_py, py::arg("files"),
           "[(xet_hash, dst_ptr, size), ...] through one pipeline; returns one stats dict per file "
           "(chunk_lens: uint32 chunk sizes in file order)")
      .def("term_shapes", [](DeviceXetPull& self, const std::string& hex) {
             std::vector<zest::TermShape> v;
             {
               py::gil_scoped_release nogil;
               v = self.term_shapes(hex);
             }
             return zest::term_shapes_py(v);
           }, py::arg("xet_hash"), "[(unpacked_length, n_chunks), ...] of the file's reconstruction terms")
      .def("pull_terms",
           [](DeviceXetPull& self, const std::vector<zest::TermJobTuple>& v, uintptr_t hashes, uintptr_t sizes,
              bool repair) {
             const auto jobs = zest::term_jobs_of(v);
             std::vector<zest::TermJobResult> rs;
             {
               py::gil_scoped_release nogil;
               rs = self.pull_terms(jobs, reinterpret_cast<uint8_t*>(hashes), reinterpret_cast<uint64_t*>(sizes),
                                    repair);
             }
             return zest::term_results_py(rs);
           },
           py::arg("jobs"), py::arg("hashes_ptr"), py::arg("sizes_ptr") = 0, py::arg("repair") = false,
           "[(xet_hash, t0, t1, dst_ptr, chunk0), ...]: fetch term ranges, GPU decode + chunk-hash them into "
           "place (hashes/sizes: device tables indexed by chunk); consecutive chunk indices required")
      .def("settle", [](DeviceXetPull& self, const std::string& hex, bool ok) {
             py::gil_scoped_release nogil;
             return self.settle(hex, ok);
           }, py::arg("xet_hash"), py::arg("ok"), "publish (ok) or drop the file's quarantined runs")
      .def("stats_json", &DeviceXetPull::stats_json)
      .def_property_readonly("staging_bytes", &DeviceXetPull::staging_bytes);
}
