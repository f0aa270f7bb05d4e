// pybind11 face of the native device-direct pull (csrc/gpurt/device_pull.{h,cpp}): fetch a Xet
// file's terms through the cache -> P2P -> CDN waterfall into pinned staging and decode + BLAKE3 +
// Merkle-verify them on the GPU into caller-provided HBM.  North-star path for
// `zest_amd.pull(..., device=...)` and the owner fetch of `parallel.swarm_pull`.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../gpurt/device_pull.h"
#include "hub.h"
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
  // This module links its own copy of the host core: the memory origin that DeviceXetPull's fetches
  // read must be registered here (zest_amd.ops.mem_origin_add registers in _core and _hip).
  m.def("mem_origin_add", [](std::vector<std::string> hexes, std::vector<uint64_t> starts, std::vector<uintptr_t> ptrs,
                             std::vector<uint64_t> lens) {
    if (starts.size() != hexes.size() || ptrs.size() != hexes.size() || lens.size() != hexes.size())
      throw std::invalid_argument("mem_origin_add: lists of different lengths");
    for (size_t i = 0; i < hexes.size(); ++i)
      zest::cas::mem_origin_add(hexes[i], starts[i], reinterpret_cast<const uint8_t*>(ptrs[i]), lens[i]);
    return zest::cas::mem_origin_size();
  }, py::arg("xorb_hexes"), py::arg("url_starts"), py::arg("ptrs"), py::arg("lens"));
  m.def("mem_origin_clear", &zest::cas::mem_origin_clear);
  m.def("mem_origin_size", &zest::cas::mem_origin_size);

  py::class_<DeviceXetPull>(m, "DeviceXetPull", "Xet pull with GPU ingest + verification into HBM")
      .def(py::init([](const std::string& repo, const std::string& revision, const std::string& repo_type, bool p2p,
                       std::vector<std::string> peers, std::optional<std::string> tracker, bool dht,
                       std::vector<std::string> boot, int device, size_t staging, int threads, int slots) {
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
             o.slots = slots;
             // Authentication talks HTTP: release the GIL (the hub may be served from this process).
             py::gil_scoped_release nogil;
             return new DeviceXetPull(o);
           }),
           py::arg("repo"), py::arg("revision") = "main", py::arg("repo_type") = "model", py::arg("p2p") = true,
           py::arg("peers") = std::vector<std::string>{}, py::arg("tracker") = std::nullopt, py::arg("dht") = true,
           py::arg("dht_bootstrap") = std::vector<std::string>{}, py::arg("device") = 0,
           py::arg("staging_bytes") = size_t(1) << 30, py::arg("threads") = 16, py::arg("slots") = 0)
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
      .def("term_keys", [](DeviceXetPull& self, const std::string& hex) {
             std::vector<zest::TermKey> v;
             {
               py::gil_scoped_release nogil;
               v = self.term_keys(hex);
             }
             return zest::term_keys_py(v);
           }, py::arg("xet_hash"), "[(xorb_hex, chunk_start, chunk_end), ...] of the file's reconstruction terms")
      .def("cached_terms", [](DeviceXetPull& self, std::vector<std::string> hexes, std::vector<uint32_t> starts,
                              std::vector<uint32_t> ends) {
             std::vector<uint8_t> v;
             {
               py::gil_scoped_release nogil;
               v = self.cached_terms(hexes, starts, ends);
             }
             return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
           }, py::arg("hexes"), py::arg("starts"), py::arg("ends"),
           "one byte per term: 1 when the local xorb cache covers its chunk range (planner possession check)")
      .def("reset_reconstructions", &DeviceXetPull::reset_reconstructions, "forget cached reconstructions (between pulls)")
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
      .def("submit_terms",
           [](DeviceXetPull& self, const std::vector<zest::TermJobTuple>& v, uintptr_t hashes, uintptr_t sizes) {
             const auto jobs = zest::term_jobs_of(v);
             py::gil_scoped_release nogil;
             return self.submit_terms(jobs, reinterpret_cast<uint8_t*>(hashes), reinterpret_cast<uint64_t*>(sizes));
           },
           py::arg("jobs"), py::arg("hashes_ptr"), py::arg("sizes_ptr") = 0,
           "pull_terms as one item of the persistent streaming pipeline (no drain between items): returns a "
           "ticket at once; wait_item(ticket) collects it")
      .def("wait_item",
           [](DeviceXetPull& self, uint64_t ticket) {
             DeviceXetPull::ItemResult r;
             {
               py::gil_scoped_release nogil;
               r = self.wait_item(ticket);
             }
             return py::make_tuple(r.err, r.err.empty() ? zest::term_results_py(r.results) : py::list(), r.event);
           },
           py::arg("ticket"),
           "(error, results, event): blocks until the item's kernels are queued (or it failed); event is a "
           "hipEvent_t (int) completing with them -- order exchanges after it with stream_wait_event")
      .def("item_error",
           [](DeviceXetPull& self, uint64_t ticket) {
             py::gil_scoped_release nogil;
             return self.item_error(ticket);
           },
           py::arg("ticket"), "the item's device decode error word (0 = clean); waits for its kernels")
      .def("stream_reset",
           [](DeviceXetPull& self, bool cancel) {
             py::gil_scoped_release nogil;
             self.stream_reset(cancel);
           },
           py::arg("cancel") = false,
           "wait for every submitted item and forget them (between pulls); cancel: abandon the ones still "
           "fetching first")
      .def("order_after", [](DeviceXetPull& self, uintptr_t event) { self.order_after(event); }, py::arg("event"),
           "queue everything this pipeline does from now on behind the caller's hipEvent_t (int)")
      .def("settle", [](DeviceXetPull& self, const std::string& hex, bool ok) {
             py::gil_scoped_release nogil;
             return self.settle(hex, ok);
           }, py::arg("xet_hash"), py::arg("ok"), "publish (ok) or drop the file's quarantined runs")
      .def("sibling", [](const DeviceXetPull& self, size_t staging, int slots) { return self.sibling(staging, slots); },
           py::arg("staging_bytes") = 0, py::arg("slots") = 0,
           "a second pipeline (own streams + staging) sharing this one's Xet session, caches and settle book")
      .def("flush_cache_writes", [](DeviceXetPull& self) {
             py::gil_scoped_release nogil;
             self.flush_cache_writes();
           }, "wait for the write-behind xorb cache queue")
      .def("cache_writer_json", &DeviceXetPull::cache_writer_json)
      .def("timeline_json", &DeviceXetPull::timeline_json)
      .def("stats_json", &DeviceXetPull::stats_json)
      .def_property_readonly("staging_bytes", &DeviceXetPull::staging_bytes);
}
