// pybind11 bindings for the zest host core (`zest_amd._core`).
#include <thread>
#include <atomic>
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <cstring>

#include "blake3.h"
#include "cdc.h"
#include "common.h"
#include "lz4.h"
#include "xet_hash.h"
#include "xorb.h"
#include "bind_extra.h"

namespace py = pybind11;
using namespace zest;

namespace {

ByteSpan span_of(const py::buffer& b) {
  py::buffer_info info = b.request();
  return ByteSpan(static_cast<const uint8_t*>(info.ptr), size_t(info.size) * size_t(info.itemsize));
}

py::bytes to_bytes(const uint8_t* p, size_t n) { return py::bytes(reinterpret_cast<const char*>(p), n); }
py::bytes to_bytes(const Bytes& b) { return to_bytes(b.data(), b.size()); }
py::bytes to_bytes(const xet::Hash& h) { return to_bytes(h.data(), 32); }

xet::Hash hash_of(const py::bytes& b) {
  std::string s = b;
  if (s.size() != 32) throw Error("InvalidHash", "hash must be 32 bytes");
  xet::Hash h;
  std::memcpy(h.data(), s.data(), 32);
  return h;
}

std::vector<xet::HashSize> leaves_of(const py::list& l) {
  std::vector<xet::HashSize> out;
  out.reserve(l.size());
  for (auto item : l) {
    auto t = item.cast<py::tuple>();
    out.push_back({hash_of(t[0].cast<py::bytes>()), t[1].cast<uint64_t>()});
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_core, m) {
  m.doc() = "zest MI355X-native framework: host core (C++17)";
  static py::exception<Error> zerr(m, "ZestError");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const Error& e) {
      py::handle cls = zerr;
      py::object exc = cls(py::str(e.what()));
      exc.attr("code") = e.code();
      PyErr_SetObject(zerr.ptr(), exc.ptr());
    }
  });

  // ---------------- BLAKE3 ----------------
  m.def("blake3", [](py::buffer b) {
    ByteSpan s = span_of(b);
    uint8_t out[32];
    {
      py::gil_scoped_release nogil;
      blake3::hash(s.data, s.size, out);
    }
    return to_bytes(out, 32);
  });
  m.def("blake3_keyed", [](py::bytes key, py::buffer b) {
    std::string k = key;
    if (k.size() != 32) throw Error("InvalidKey", "key must be 32 bytes");
    ByteSpan s = span_of(b);
    uint8_t out[32];
    {
      py::gil_scoped_release nogil;
      blake3::keyed_hash(reinterpret_cast<const uint8_t*>(k.data()), s.data, s.size, out);
    }
    return to_bytes(out, 32);
  });
  m.def("blake3_backend", &blake3::simd_backend);
  m.def("blake3_force_backend", [](const std::string& n) { return blake3::force_backend(n.c_str()); });

  // ---------------- Xet hashing ----------------
  m.attr("DATA_KEY") = to_bytes(xet::kDataKey, 32);
  m.attr("INTERNAL_NODE_KEY") = to_bytes(xet::kInternalNodeKey, 32);
  m.def("chunk_hash", [](py::buffer b) {
    ByteSpan s = span_of(b);
    xet::Hash h;
    {
      py::gil_scoped_release nogil;
      h = xet::chunk_hash(s.data, s.size);
    }
    return to_bytes(h);
  });
  m.def("internal_node_hash", [](py::buffer b) {
    ByteSpan s = span_of(b);
    return to_bytes(xet::internal_node_hash(s.data, s.size));
  });
  m.def("xet_hex", [](py::bytes b) { return xet::to_hex(hash_of(b)); });
  m.def("from_xet_hex", [](const std::string& s) { return to_bytes(xet::from_hex(s)); });
  m.def("bytewise_hex", [](py::buffer b) {
    ByteSpan s = span_of(b);
    return xet::to_bytewise_hex(s.data, s.size);
  });
  m.def("merkle_root", [](py::list l) { return to_bytes(xet::merkle_root(leaves_of(l))); });
  m.def("file_hash", [](py::list l) { return to_bytes(xet::file_hash(leaves_of(l))); });
  m.def("file_hash_from_root", [](py::bytes root) { return to_bytes(xet::file_hash_from_root(hash_of(root), false)); });
  m.def("next_merge_cut", [](py::list l) {
    auto v = leaves_of(l);
    return xet::next_merge_cut(v.data(), v.size());
  });
  m.def("chunk_ends", [](py::buffer b, size_t target) {
    ByteSpan s = span_of(b);
    xet::CdcParams p;
    p.target = target;
    p.min_size = target / 8;
    p.max_size = target * 2;
    std::vector<uint64_t> e;
    {
      py::gil_scoped_release nogil;
      e = xet::chunk_ends(s.data, s.size, p);
    }
    return e;
  }, py::arg("data"), py::arg("target") = 65536);
  m.def("select_boundaries", [](py::buffer cand, uint64_t n, size_t mn, size_t mx) {
    py::buffer_info bi = cand.request();
    if (bi.itemsize != 8) throw Error("InvalidArgument", "candidates must be uint64");
    return xet::select_boundaries(static_cast<const uint64_t*>(bi.ptr), size_t(bi.size), n, mn, mx);
  });
  // Greedy xorb packing (xorb <= max_bytes serialized, <= max_chunks chunks), as an uploader
  // does: returns the xorb index of every chunk given its serialized size (header + payload).
  m.def("plan_xorbs", [](py::buffer ser_sizes, uint64_t max_bytes, uint32_t max_chunks) {
    py::buffer_info bi = ser_sizes.request();
    if (bi.itemsize != 8) throw Error("InvalidArgument", "sizes must be uint64");
    const uint64_t* s = static_cast<const uint64_t*>(bi.ptr);
    const size_t n = size_t(bi.size);
    py::array_t<int64_t> out(n);
    auto o = out.mutable_unchecked<1>();
    int64_t x = 0;
    uint64_t bytes = 0;
    uint32_t cnt = 0;
    for (size_t i = 0; i < n; ++i) {
      if (cnt > 0 && (bytes + s[i] > max_bytes || cnt + 1 > max_chunks)) {
        ++x;
        bytes = 0;
        cnt = 0;
      }
      o(i) = x;
      bytes += s[i];
      ++cnt;
    }
    return out;
  });
  m.def("gear_window_hash", [](py::buffer b, size_t i) { return xet::gear_window_hash(span_of(b).data, i); });
  // Whole-buffer Xet file hash (CDC + chunk hashes + Merkle + salt) — `zest` equivalent of
  // hf_xet.hash_files for in-memory data.
  m.def("xet_file_hash", [](py::buffer b) {
    ByteSpan s = span_of(b);
    xet::Hash h;
    {
      py::gil_scoped_release nogil;
      auto ends = xet::chunk_ends(s.data, s.size);
      std::vector<xet::HashSize> leaves;
      leaves.reserve(ends.size());
      uint64_t prev = 0;
      for (uint64_t e : ends) {
        leaves.push_back({xet::chunk_hash(s.data + prev, e - prev), e - prev});
        prev = e;
      }
      h = xet::file_hash(leaves);
    }
    return to_bytes(h);
  });

  // Xet file hash with the chunk boundaries given (uint32 chunk sizes, e.g. the ones the owner of a
  // swarm piece parsed from the xorb headers): chunk hashes + Merkle + salt, no CDC pass.  Wrong
  // boundaries give a different hash, so they need no trust.
  m.def("xet_file_hash_lens", [](py::buffer b, py::buffer lens_b) {
    ByteSpan s = span_of(b);
    ByteSpan lb = span_of(lens_b);
    if (lb.size % 4) throw Error("InvalidArgument", "chunk lens must be uint32");
    const size_t n = lb.size / 4;
    std::vector<uint32_t> lens(n);
    std::memcpy(lens.data(), lb.data, lb.size);
    uint64_t total = 0;
    for (uint32_t l : lens) total += l;
    if (total != s.size) return py::bytes();  // boundaries do not cover the buffer: no hash
    xet::Hash h;
    {
      py::gil_scoped_release nogil;
      std::vector<xet::HashSize> leaves(n);
      std::vector<uint64_t> off(n + 1, 0);
      for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + lens[i];
      std::atomic<size_t> next{0};
      auto work = [&]() {
        for (size_t i; (i = next.fetch_add(64)) < n;)
          for (size_t j = i; j < std::min(n, i + 64); ++j)
            leaves[j] = {xet::chunk_hash(s.data + off[j], lens[j]), lens[j]};
      };
      std::vector<std::thread> ts;
      const size_t nt = std::min<size_t>(8, std::max<size_t>(1, n / 64));
      for (size_t t = 1; t < nt; ++t) ts.emplace_back(work);
      work();
      for (auto& t : ts) t.join();
      h = xet::file_hash(leaves);
    }
    return to_bytes(h);
  });

  // ---------------- LZ4 / BG4 ----------------
  m.def("xxh32", [](py::buffer b, uint32_t seed) {
    ByteSpan s = span_of(b);
    return lz4::xxh32(s.data, s.size, seed);
  }, py::arg("data"), py::arg("seed") = 0);
  m.def("lz4_compress_frame", [](py::buffer b) {
    ByteSpan s = span_of(b);
    Bytes out;
    {
      py::gil_scoped_release nogil;
      out = lz4::compress_frame(s.data, s.size);
    }
    return to_bytes(out);
  });
  m.def("lz4_decompress_frame", [](py::buffer b, size_t expected) {
    ByteSpan s = span_of(b);
    Bytes out;
    {
      py::gil_scoped_release nogil;
      out = lz4::decompress_frame(s.data, s.size, expected);
    }
    return to_bytes(out);
  }, py::arg("data"), py::arg("expected") = 0);
  m.def("lz4_compress_block", [](py::buffer b) {
    ByteSpan s = span_of(b);
    Bytes out(lz4::block_bound(s.size));
    size_t n = lz4::compress_block(s.data, s.size, out.data(), out.size());
    return to_bytes(out.data(), n);
  });
  m.def("lz4_decompress_block", [](py::buffer b, size_t cap) {
    ByteSpan s = span_of(b);
    Bytes out(cap);
    size_t n = lz4::decompress_block(s.data, s.size, out.data(), 0, cap);
    return to_bytes(out.data(), n);
  });
  m.def("bg4_split", [](py::buffer b) {
    ByteSpan s = span_of(b);
    Bytes out(s.size);
    bg4::split(s.data, s.size, out.data());
    return to_bytes(out);
  });
  m.def("bg4_join", [](py::buffer b) {
    ByteSpan s = span_of(b);
    Bytes out(s.size);
    bg4::join(s.data, s.size, out.data());
    return to_bytes(out);
  });
  m.def("compress_chunk", [](py::buffer b, const std::string& policy) {
    ByteSpan s = span_of(b);
    xet::CompressionPolicy p = policy == "none" ? xet::CompressionPolicy::None
                               : policy == "lz4" ? xet::CompressionPolicy::LZ4
                               : policy == "bg4" ? xet::CompressionPolicy::BG4
                                                 : xet::CompressionPolicy::Auto;
    Bytes out;
    xet::Scheme sc;
    {
      py::gil_scoped_release nogil;
      sc = xet::compress_chunk(s.data, s.size, p, out);
    }
    return py::make_tuple(int(sc), to_bytes(out));
  }, py::arg("data"), py::arg("policy") = "auto");
  m.def("decompress_chunk", [](int scheme, py::buffer b, size_t ulen) {
    ByteSpan s = span_of(b);
    Bytes out(ulen);
    xet::decompress_chunk(xet::Scheme(scheme), s.data, s.size, out.data(), ulen);
    return to_bytes(out);
  });

  // ---------------- Xorb ----------------
  m.def("index_chunks", [](py::buffer b) {
    ByteSpan s = span_of(b);
    auto idx = xet::index_chunks(s.data, s.size);
    py::list out;
    for (auto& e : idx)
      out.append(py::make_tuple(e.header_off, e.clen, int(e.scheme), e.ulen, e.unpacked_off));
    return out;
  });
  // Host header walk over a staging span of fetched runs: the same records and error words as the
  // device kernel k_index_terms (csrc/gpu/ingest.hip), for callers whose bytes are in host memory
  // anyway (the pull engine's origin): a pointer chase runs at host DRAM latency instead of HBM
  // latency, and the GPU then only places and hashes.  terms: TERM_DTYPE records (40 B), out:
  // CHUNK_DTYPE records (32 B) for n_out chunks (gaps between terms become zero no-op records).
  // Returns 0, or code << 32 | term for the first bad term (codes as ZG_ERR_*).
  m.def("index_runs", [](uintptr_t span, uint64_t span_len, uintptr_t terms, int n_terms, uintptr_t out,
                         uint64_t n_out) -> uint64_t {
    struct Term {
      uint64_t src, src_len, dst;
      uint32_t chunk_base, n_chunks;
      uint64_t ulen;
    };
    struct Chunk {
      uint64_t src, dst;
      uint32_t clen, ulen, scheme, term;
    };
    static_assert(sizeof(Term) == 40 && sizeof(Chunk) == 32, "TERM_DTYPE / CHUNK_DTYPE layout");
    py::gil_scoped_release nogil;
    const uint8_t* base = reinterpret_cast<const uint8_t*>(span);
    const Term* tv = reinterpret_cast<const Term*>(terms);
    Chunk* cv = reinterpret_cast<Chunk*>(out);
    std::memset(cv, 0, n_out * sizeof(Chunk));
    uint64_t first_err = 0;
    for (int t = 0; t < n_terms; ++t) {
      const Term tm = tv[t];
      uint64_t err = 0;
      if (uint64_t(tm.chunk_base) + tm.n_chunks > n_out || tm.src + tm.src_len > span_len) err = 2;  // ZG_ERR_RANGE
      uint64_t off = 0, uoff = 0;
      for (uint32_t c = 0; c < tm.n_chunks && !err; ++c) {
        if (off + 8 > tm.src_len) {
          err = 3;  // ZG_ERR_COUNT
          break;
        }
        const uint8_t* h = base + tm.src + off;
        const uint32_t clen = uint32_t(h[1]) | uint32_t(h[2]) << 8 | uint32_t(h[3]) << 16;
        const uint32_t scheme = h[4];
        const uint32_t ulen = uint32_t(h[5]) | uint32_t(h[6]) << 8 | uint32_t(h[7]) << 16;
        if (h[0] != 0 || scheme > 2 || (scheme == 0 && clen != ulen)) err = 1;  // ZG_ERR_HEADER
        else if (off + 8 + clen > tm.src_len || (tm.ulen != 0 && uoff + ulen > tm.ulen)) err = 2;
        else if (ulen > 128u * 1024u) err = 7;  // ZG_ERR_CAPACITY
        if (err) break;
        cv[tm.chunk_base + c] = Chunk{tm.src + off + 8, tm.dst + uoff, clen, ulen, scheme, uint32_t(t)};
        off += 8 + clen;
        uoff += ulen;
      }
      if (err) {  // the term's records stay zero (no-ops), as the device kernel leaves them
        if (uint64_t(tm.chunk_base) + tm.n_chunks <= n_out)
          std::memset(cv + tm.chunk_base, 0, size_t(tm.n_chunks) * sizeof(Chunk));
      } else if (off != tm.src_len || (tm.ulen != 0 && uoff != tm.ulen)) {
        err = 3;
      }
      if (err && !first_err) first_err = err << 32 | uint32_t(t);
    }
    return first_err;
  }, py::arg("span"), py::arg("span_len"), py::arg("terms"), py::arg("n_terms"), py::arg("out"), py::arg("n_out"));
  m.def("parse_footer", [](py::buffer b) -> py::object {
    ByteSpan s = span_of(b);
    size_t st = 0;
    auto f = xet::parse_footer(s.data, s.size, &st);
    if (!f) return py::none();
    py::dict d;
    d["xorb_hash"] = to_bytes(f->xorb_hash);
    py::list hs;
    for (auto& h : f->chunk_hashes) hs.append(to_bytes(h));
    d["chunk_hashes"] = hs;
    d["chunk_boundaries"] = f->chunk_boundaries;
    d["unpacked_offsets"] = f->unpacked_offsets;
    d["footer_start"] = st;
    return d;
  });
  m.def("extract_chunk_range", [](py::buffer b, uint32_t start, uint32_t end, bool with_hashes) {
    ByteSpan s = span_of(b);
    Bytes out;
    std::vector<xet::HashSize> hs;
    {
      py::gil_scoped_release nogil;
      xet::extract_chunk_range(s.data, s.size, start, end, out, with_hashes ? &hs : nullptr);
    }
    if (!with_hashes) return py::object(to_bytes(out));
    py::list l;
    for (auto& h : hs) l.append(py::make_tuple(to_bytes(h.hash), h.size));
    return py::object(py::make_tuple(to_bytes(out), l));
  }, py::arg("data"), py::arg("start"), py::arg("end"), py::arg("with_hashes") = false);
  m.def("verify_xorb", [](py::buffer b, py::object expected) {
    ByteSpan s = span_of(b);
    if (expected.is_none()) {
      py::gil_scoped_release nogil;
      xet::verify_xorb(s.data, s.size, nullptr);
    } else {
      xet::Hash h = hash_of(expected.cast<py::bytes>());
      py::gil_scoped_release nogil;
      xet::verify_xorb(s.data, s.size, &h);
    }
  }, py::arg("data"), py::arg("expected") = py::none());

  py::class_<xet::XorbBuilder>(m, "XorbBuilder")
      .def(py::init([](const std::string& policy) {
             xet::CompressionPolicy p = policy == "none" ? xet::CompressionPolicy::None
                                        : policy == "lz4" ? xet::CompressionPolicy::LZ4
                                        : policy == "bg4" ? xet::CompressionPolicy::BG4
                                                          : xet::CompressionPolicy::Auto;
             return new xet::XorbBuilder(p);
           }),
           py::arg("policy") = "auto")
      .def("fits", &xet::XorbBuilder::fits)
      .def("add_chunk", [](xet::XorbBuilder& self, py::buffer b) {
        ByteSpan s = span_of(b);
        py::gil_scoped_release nogil;
        return self.add_chunk(s.data, s.size);
      })
      .def("num_chunks", &xet::XorbBuilder::num_chunks)
      .def("serialized_size", &xet::XorbBuilder::serialized_size)
      .def("unpacked_size", &xet::XorbBuilder::unpacked_size)
      .def("hash", [](const xet::XorbBuilder& self) { return to_bytes(self.hash()); })
      .def("chunk_hashes", [](const xet::XorbBuilder& self) {
        py::list l;
        for (auto& h : self.chunk_hashes()) l.append(to_bytes(h));
        return l;
      })
      .def("chunk_ulens", &xet::XorbBuilder::chunk_ulens)
      .def("chunk_boundaries", &xet::XorbBuilder::chunk_boundaries)
      .def("serialize", [](const xet::XorbBuilder& self, bool footer) { return to_bytes(self.serialize(footer)); },
           py::arg("with_footer") = true)
      .def("clear", &xet::XorbBuilder::clear);

  bind_extra(m);
}
