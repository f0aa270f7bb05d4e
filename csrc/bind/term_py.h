// pybind11 helpers of the term-range fetch API (csrc/core/term_jobs.h), shared by the host module
// (_core.HostXetFetcher) and the HIP module (_hip.DeviceXetPull).
#pragma once

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <string>
#include <tuple>
#include <vector>

#include "term_jobs.h"

namespace zest {

using TermJobTuple = std::tuple<std::string, uint32_t, uint32_t, uintptr_t, uint64_t>;

// Python face of the term-range API, shared by HostXetFetcher and DeviceXetPull: jobs are
// (xet_hash, t0, t1, dst_ptr, chunk0) tuples; results are dicts.
inline std::vector<TermJob> term_jobs_of(const std::vector<TermJobTuple>& v) {
  std::vector<TermJob> jobs;
  jobs.reserve(v.size());
  for (const auto& j : v) jobs.push_back({std::get<0>(j), std::get<1>(j), std::get<2>(j), std::get<3>(j), std::get<4>(j)});
  return jobs;
}

inline pybind11::list term_results_py(const std::vector<TermJobResult>& rs) {
  pybind11::list out;
  for (const auto& r : rs) {
    pybind11::dict d;
    d["chunk_lens"] = pybind11::bytes(reinterpret_cast<const char*>(r.chunk_lens.data()), 4 * r.chunk_lens.size());
    d["fetched"] = r.fetched;
    d["from_peer"] = r.from_peer;
    d["from_cdn"] = r.from_cdn;
    d["from_cache"] = r.from_cache;
    out.append(d);
  }
  return out;
}

inline pybind11::list term_shapes_py(const std::vector<TermShape>& v) {
  pybind11::list out;
  for (const auto& t : v) out.append(pybind11::make_tuple(t.ulen, t.nchunks));
  return out;
}

inline pybind11::list term_keys_py(const std::vector<TermKey>& v) {
  pybind11::list out;
  for (const auto& t : v) out.append(pybind11::make_tuple(t.hex, t.start, t.end));
  return out;
}

}  // namespace zest
