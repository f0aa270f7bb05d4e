// pybind11 bindings for the native control plane: bencode, BT wire, BEP XET, SHA-1 info-hash,
// tracker, DHT, BT server / peer client, xorb cache, pull and the synthetic benchmark.
// Submodules of `zest_amd._core` so Python code reads `_core.bencode.decode(...)` etc.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <sstream>
#include <thread>
#include <atomic>

#include "swarm.h"
#include "bridge.h"
#include "downloader.h"
#include "bench.h"
#include "bencode.h"
#include "bind_extra.h"
#include "bt_peer.h"
#include "bt_server.h"
#include "bt_wire.h"
#include "config.h"
#include "dht.h"
#include "http.h"
#include "hub.h"
#include "pull.h"
#include "sha1.h"
#include "storage.h"
#include "term_jobs.h"
#include "term_py.h"
#include "trace.h"
#include "tracker.h"
#include "xet_hash.h"

namespace py = pybind11;
using namespace zest;

namespace {

py::bytes pyb(const void* p, size_t n) { return py::bytes(static_cast<const char*>(p), n); }
py::bytes pyb(const Bytes& b) { return pyb(b.data(), b.size()); }
py::bytes pyb(std::string_view s) { return pyb(s.data(), s.size()); }
py::bytes pyb(ByteSpan s) { return pyb(s.data, s.size); }

template <size_t N>
std::array<uint8_t, N> arr_of(const py::bytes& b, const char* what) {
  std::string s = b;
  if (s.size() != N) throw Error("InvalidLength", std::string(what) + " must be " + std::to_string(N) + " bytes");
  std::array<uint8_t, N> a;
  std::memcpy(a.data(), s.data(), N);
  return a;
}

// ---- bencode <-> Python
py::object bdecode_ref(bencode::Ref r) {
  switch (r.type()) {
    case bencode::Type::Int:
      return py::int_(r.as_int());
    case bencode::Type::Str:
      return pyb(r.as_str());
    case bencode::Type::List: {
      py::list l;
      for (auto& c : r.children()) l.append(bdecode_ref(c));
      return l;
    }
    case bencode::Type::Dict: {
      py::dict d;
      for (auto& c : r.children()) d[pyb(c.key())] = bdecode_ref(c);
      return d;
    }
  }
  return py::none();
}

void bencode_obj(bencode::Encoder& e, const py::handle& o) {
  if (py::isinstance<py::bool_>(o)) {
    e.integer(o.cast<bool>() ? 1 : 0);
  } else if (py::isinstance<py::int_>(o)) {
    e.integer(o.cast<int64_t>());
  } else if (py::isinstance<py::bytes>(o)) {
    e.str(std::string(o.cast<py::bytes>()));
  } else if (py::isinstance<py::str>(o)) {
    e.str(o.cast<std::string>());
  } else if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    e.begin_list();
    for (auto item : o) bencode_obj(e, item);
    e.end();
  } else if (py::isinstance<py::dict>(o)) {
    std::vector<std::pair<std::string, py::handle>> items;
    for (auto kv : o.cast<py::dict>()) {
      std::string k = py::isinstance<py::bytes>(kv.first) ? std::string(kv.first.cast<py::bytes>())
                                                         : kv.first.cast<std::string>();
      items.emplace_back(std::move(k), kv.second);
    }
    std::sort(items.begin(), items.end(), [](auto& a, auto& b) { return a.first < b.first; });
    e.begin_dict();
    for (auto& [k, v] : items) {
      e.key(k);
      bencode_obj(e, v);
    }
    e.end();
  } else {
    throw Error("InvalidFormat", "cannot bencode object of this type");
  }
}

py::dict xet_msg_dict(const bep_xet::Message& m) {
  py::dict d;
  d["type"] = int(m.type);
  d["request_id"] = m.request_id;
  switch (m.type) {
    case bep_xet::kChunkRequest:
      d["hash"] = pyb(m.hash.data(), 32);
      d["range_start"] = m.range_start;
      d["range_end"] = m.range_end;
      break;
    case bep_xet::kChunkResponse:
      d["chunk_offset"] = m.chunk_offset;
      d["data"] = pyb(m.data);
      break;
    case bep_xet::kChunkNotFound:
      d["hash"] = pyb(m.hash.data(), 32);
      break;
    case bep_xet::kChunkError:
      d["error_code"] = m.error_code;
      d["message"] = pyb(m.data);
      break;
  }
  return d;
}

std::vector<std::string> addr_strs(const std::vector<net::Addr>& v) {
  std::vector<std::string> out;
  for (auto& a : v) out.push_back(a.str());
  return out;
}

// Python-owned BT seeder: a cache + registry + server bundled together.
struct PySeeder {
  Config cfg;
  storage::XorbRegistry registry;
  std::unique_ptr<storage::XorbCache> cache;
  std::unique_ptr<bt::BtServer> server;
  PySeeder(int port, const std::string& fault) : cfg(Config::from_env()) {
    registry.scan(cfg);
    cache = std::make_unique<storage::XorbCache>(cfg, &registry);
    server = std::make_unique<bt::BtServer>(cfg, cache.get(), bt::PieceProvider{}, port);
    if (!fault.empty()) server->set_fault(bt::FaultSpec::parse(fault));
    server->start();
  }
  ~PySeeder() { server->stop(); }
};

}  // namespace

// In-memory host fetch of Xet files (see HostXetFetcher binding below).
class HostXetFetcher {
 public:
  HostXetFetcher(const std::string& repo, const std::string& revision, const std::string& repo_type, bool p2p,
                 std::vector<std::string> peers, std::optional<std::string> tracker, bool dht,
                 std::vector<std::string> boot, int concurrency)
      : cfg_(Config::from_env()) {
    registry_.scan(cfg_);
    cache_ = std::make_unique<storage::XorbCache>(cfg_, &registry_);
    std::vector<net::Addr> b;
    for (auto& x : boot) b.push_back(net::Addr::parse(x, 6881));
    swarm_ = std::make_unique<SwarmDownloader>(cfg_, std::move(tracker), p2p, dht && p2p, b);
    for (auto& p : peers) swarm_->add_direct_peer(net::Addr::parse(p, 6881));
    bridge_ = std::make_unique<XetBridge>(cfg_, cache_.get(), swarm_.get());
    bridge_->authenticate(repo, repo_type, revision);
    threads_ = concurrency > 0 ? concurrency : int(cfg_.concurrency);
    dl_ = std::make_unique<ParallelDownloader>(*bridge_, threads_);
    recs_ = std::make_unique<ReconCache>(*bridge_);
  }
  // Term-range API of the term-sharded swarm pull (csrc/core/term_jobs.h).
  std::vector<TermShape> shapes(const std::string& hex) { return recs_->shapes(hex); }
  std::vector<TermKey> term_keys(const std::string& hex) { return recs_->keys(hex); }
  std::vector<uint8_t> cached_terms(const std::vector<std::string>& hexes, const std::vector<uint32_t>& starts,
                                    const std::vector<uint32_t>& ends) {
    return zest::cached_terms(*cache_, hexes, starts, ends, threads_);
  }
  void reset_reconstructions() { recs_->clear(); }
  std::vector<TermJobResult> fetch_terms(const std::vector<TermJob>& jobs, uint8_t* hashes, bool repair) {
    return fetch_terms_host(*bridge_, *recs_, book_, jobs, hashes, threads_, repair);
  }
  size_t settle(const std::string& hex, bool ok) { return book_.settle(*bridge_, hex, ok); }
  std::vector<FileResult> fetch(const std::vector<std::tuple<std::string, uintptr_t, uint64_t>>& files) {
    std::vector<FileResult> out(files.size());
    std::vector<std::string> errs(files.size());
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < files.size();) {
        try {
          out[i] = dl_->reconstruct_to_memory(std::get<0>(files[i]), reinterpret_cast<uint8_t*>(std::get<1>(files[i])),
                                              std::get<2>(files[i]), true);
        } catch (const std::exception& e) {
          errs[i] = e.what();
        }
      }
    };
    std::vector<std::thread> ts;
    for (size_t t = 1; t < std::min<size_t>(4, files.size()); ++t) ts.emplace_back(work);
    work();
    for (auto& t : ts) t.join();
    for (size_t i = 0; i < files.size(); ++i)
      if (!errs[i].empty()) throw Error("DownloadFailed", std::get<0>(files[i]) + ": " + errs[i]);
    return out;
  }
  std::string stats_json() const { return bridge_->stats_json(); }

 private:
  Config cfg_;
  storage::XorbRegistry registry_;
  std::unique_ptr<storage::XorbCache> cache_;
  std::unique_ptr<SwarmDownloader> swarm_;
  std::unique_ptr<XetBridge> bridge_;
  std::unique_ptr<ParallelDownloader> dl_;
  std::unique_ptr<ReconCache> recs_;
  SettleBook book_;
  int threads_ = 16;
};


void bind_extra(py::module_& m) {
  // ---------------- bencode ----------------
  auto mb = m.def_submodule("bencode", "BEP 3 bencode (strict decoder, canonical encoder)");
  mb.def("decode", [](py::bytes b) {
    std::string s = b;
    bencode::Document doc;
    doc.parse(s);
    return bdecode_ref(doc.root());
  });
  mb.def("decode_prefix", [](py::bytes b) {
    std::string s = b;
    bencode::Document doc;
    size_t used = doc.parse(s);
    return py::make_tuple(bdecode_ref(doc.root()), used);
  });
  mb.def("encode", [](py::object o) {
    std::string out;
    bencode::Encoder e(out);
    bencode_obj(e, o);
    return pyb(out);
  });
  mb.def("roundtrip", [](py::bytes b) {
    std::string s = b;
    bencode::Document doc;
    doc.parse(s);
    return pyb(bencode::encode(doc.root()));
  });

  // ---------------- SHA-1 / peer id ----------------
  m.def("sha1", [](py::bytes b) {
    std::string s = b;
    auto d = Sha1::hash(s.data(), s.size());
    return pyb(d.data(), d.size());
  });
  m.def("sha1_backend", []() { return std::string(Sha1::backend()); });
  m.def("info_hash", [](py::bytes xorb_hash) {
    auto h = arr_of<32>(xorb_hash, "xorb hash");
    auto d = peer_id::info_hash(h.data());
    return pyb(d.data(), d.size());
  });
  m.def("generate_peer_id", []() {
    auto p = peer_id::generate();
    return pyb(p.data(), p.size());
  });
  m.attr("CLIENT_PREFIX") = std::string(peer_id::kClientPrefix);
  m.attr("VERSION") = std::string(kVersion);

  // ---------------- BT wire ----------------
  auto mw = m.def_submodule("bt", "BitTorrent wire protocol (BEP 3 + BEP 10)");
  mw.attr("HANDSHAKE_LEN") = bt::kHandshakeLen;
  mw.attr("MAX_MESSAGE") = bt::kMaxMessage;
  mw.def("handshake", [](py::bytes ih, py::bytes pid) {
    Bytes out;
    bt::write_handshake(out, arr_of<20>(ih, "info_hash"), arr_of<20>(pid, "peer_id"));
    return pyb(out);
  });
  mw.def("parse_handshake", [](py::bytes b) {
    std::string s = b;
    if (s.size() < bt::kHandshakeLen) throw Error("UnexpectedEnd", "handshake needs 68 bytes");
    auto h = bt::parse_handshake(reinterpret_cast<const uint8_t*>(s.data()));
    py::dict d;
    d["reserved"] = pyb(h.reserved.data(), 8);
    d["info_hash"] = pyb(h.info_hash.data(), 20);
    d["peer_id"] = pyb(h.peer_id.data(), 20);
    d["bep10"] = h.supports_bep10();
    return d;
  });
  mw.def("message", [](int id, py::bytes payload) {
    std::string p = payload;
    Bytes out;
    bt::write_message(out, uint8_t(id), reinterpret_cast<const uint8_t*>(p.data()), p.size());
    return pyb(out);
  }, py::arg("id"), py::arg("payload") = py::bytes());
  mw.def("keepalive", []() {
    Bytes out;
    bt::write_keepalive(out);
    return pyb(out);
  });
  mw.def("extended", [](int ext_id, py::bytes payload) {
    std::string p = payload;
    Bytes out;
    bt::write_extended(out, uint8_t(ext_id), reinterpret_cast<const uint8_t*>(p.data()), p.size());
    return pyb(out);
  });
  mw.def("parse_message", [](py::bytes b) -> py::object {
    std::string s = b;
    bt::Message msg;
    size_t used = bt::parse_message(reinterpret_cast<const uint8_t*>(s.data()), s.size(), msg);
    if (!used) return py::none();
    py::dict d;
    d["consumed"] = used;
    d["keepalive"] = msg.keepalive;
    d["id"] = int(msg.id);
    d["payload"] = pyb(msg.payload);
    return d;
  });
  mw.def("frame_length", [](py::bytes b) {
    std::string s = b;
    return bt::frame_length(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  mw.def("parse_extended", [](py::bytes b) {
    std::string s = b;
    auto e = bt::parse_extended(ByteSpan(s));
    return py::make_tuple(int(e.ext_id), pyb(e.data));
  });
  mw.def("known_msg_id", [](int id) { return bt::known_msg_id(uint8_t(id)); });

  // ---------------- BEP XET ----------------
  auto mx = m.def_submodule("bep_xet", "ut_xet extension: chunk request/response over BT");
  mx.attr("CHUNK_REQUEST") = int(bep_xet::kChunkRequest);
  mx.attr("CHUNK_RESPONSE") = int(bep_xet::kChunkResponse);
  mx.attr("CHUNK_NOT_FOUND") = int(bep_xet::kChunkNotFound);
  mx.attr("CHUNK_ERROR") = int(bep_xet::kChunkError);
  mx.def("chunk_request", [](int ext, uint32_t rid, py::bytes hash, uint32_t a, uint32_t b) {
    Bytes out;
    auto h = arr_of<32>(hash, "hash");
    bep_xet::encode_chunk_request(out, uint8_t(ext), rid, h.data(), a, b);
    return pyb(out);
  });
  mx.def("chunk_response", [](int ext, uint32_t rid, uint32_t off, py::bytes data) {
    std::string d = data;
    Bytes out;
    bep_xet::encode_chunk_response(out, uint8_t(ext), rid, off, reinterpret_cast<const uint8_t*>(d.data()), d.size());
    return pyb(out);
  });
  mx.def("chunk_not_found", [](int ext, uint32_t rid, py::bytes hash) {
    Bytes out;
    auto h = arr_of<32>(hash, "hash");
    bep_xet::encode_chunk_not_found(out, uint8_t(ext), rid, h.data());
    return pyb(out);
  });
  mx.def("chunk_error", [](int ext, uint32_t rid, uint32_t code, std::string msg) {
    Bytes out;
    bep_xet::encode_chunk_error(out, uint8_t(ext), rid, code, msg);
    return pyb(out);
  });
  mx.def("decode", [](py::bytes b) {
    std::string s = b;
    return xet_msg_dict(bep_xet::decode(ByteSpan(s)));
  });
  mx.def("make_ext_handshake", [](uint16_t port, int id, std::string client) {
    return pyb(bep_xet::make_ext_handshake(port, uint8_t(id), client));
  }, py::arg("port"), py::arg("ut_xet_id") = 1, py::arg("client") = std::string(bep_xet::kClientVersion));
  mx.def("parse_ext_handshake", [](py::bytes b) {
    std::string s = b;
    auto c = bep_xet::parse_ext_handshake(ByteSpan(s));
    py::dict d;
    d["ut_xet"] = c.ut_xet_id;
    d["port"] = c.listen_port;
    d["client"] = c.client;
    return d;
  });

  // ---------------- tracker ----------------
  auto mt = m.def_submodule("tracker", "BEP 3 HTTP tracker client");
  mt.def("announce_url", [](std::string url, py::bytes ih, py::bytes pid, uint16_t port, std::string ev,
                            uint64_t up, uint64_t down, uint64_t left) {
    tracker::Event e = ev == "started" ? tracker::Event::Started
                       : ev == "stopped" ? tracker::Event::Stopped
                       : ev == "completed" ? tracker::Event::Completed
                                           : tracker::Event::None;
    return tracker::announce_url(url, arr_of<20>(ih, "info_hash"), arr_of<20>(pid, "peer_id"), port, e, up, down, left);
  }, py::arg("url"), py::arg("info_hash"), py::arg("peer_id"), py::arg("port"), py::arg("event") = "started",
     py::arg("uploaded") = 0, py::arg("downloaded") = 0, py::arg("left") = 0);
  mt.def("parse_announce", [](py::bytes b) {
    std::string s = b;
    auto r = tracker::parse_announce(s);
    py::dict d;
    d["interval"] = r.interval;
    d["peers"] = addr_strs(r.peers);
    return d;
  });
  mt.def("announce", [](std::string url, py::bytes ih, uint16_t port, std::string ev, int timeout_ms) {
    auto pid = peer_id::generate();
    tracker::Event e = ev == "started" ? tracker::Event::Started
                       : ev == "stopped" ? tracker::Event::Stopped
                       : ev == "completed" ? tracker::Event::Completed
                                           : tracker::Event::None;
    auto ihb = arr_of<20>(ih, "info_hash");
    tracker::AnnounceResponse r;
    {
      py::gil_scoped_release nogil;
      r = tracker::announce(url, ihb, pid, port, e, timeout_ms);
    }
    return addr_strs(r.peers);
  }, py::arg("url"), py::arg("info_hash"), py::arg("port"), py::arg("event") = "started", py::arg("timeout_ms") = 5000);
  mt.def("parse_compact_peers", [](py::bytes b, bool v6) {
    std::string s = b;
    return addr_strs(tracker::parse_compact_peers(s, v6));
  }, py::arg("data"), py::arg("v6") = false);
  mt.def("encode_compact_peer", [](std::string a) { return pyb(tracker::encode_compact_peer(net::Addr::parse(a, 0))); });

  // ---------------- DHT ----------------
  auto md = m.def_submodule("dht", "BEP 5 Kademlia DHT");
  md.def("xor_distance", [](py::bytes a, py::bytes b) {
    auto d = dht::xor_distance(arr_of<20>(a, "id"), arr_of<20>(b, "id"));
    return pyb(d.data(), 20);
  });
  md.def("bucket_index", [](py::bytes own, py::bytes other) {
    return dht::bucket_index(arr_of<20>(own, "id"), arr_of<20>(other, "id"));
  });
  md.def("random_id", []() {
    auto id = dht::random_id();
    return pyb(id.data(), 20);
  });
  md.def("build_ping", [](py::bytes tid, py::bytes own) { return pyb(dht::build_ping(std::string(tid), arr_of<20>(own, "id"))); });
  md.def("build_find_node", [](py::bytes tid, py::bytes own, py::bytes target) {
    return pyb(dht::build_find_node(std::string(tid), arr_of<20>(own, "id"), arr_of<20>(target, "target")));
  });
  md.def("build_get_peers", [](py::bytes tid, py::bytes own, py::bytes ih) {
    return pyb(dht::build_get_peers(std::string(tid), arr_of<20>(own, "id"), arr_of<20>(ih, "info_hash")));
  });
  md.def("build_announce_peer", [](py::bytes tid, py::bytes own, py::bytes ih, uint16_t port, py::bytes token, bool implied) {
    return pyb(dht::build_announce_peer(std::string(tid), arr_of<20>(own, "id"), arr_of<20>(ih, "info_hash"), port,
                                        std::string(token), implied));
  }, py::arg("tid"), py::arg("own"), py::arg("info_hash"), py::arg("port"), py::arg("token"), py::arg("implied_port") = false);
  md.def("parse_compact_nodes", [](py::bytes b) {
    std::string s = b;
    py::list out;
    for (auto& n : dht::parse_compact_nodes(s)) out.append(py::make_tuple(pyb(n.id.data(), 20), n.addr.str()));
    return out;
  });
  md.def("encode_compact_node", [](py::bytes id, std::string addr) {
    dht::NodeInfo n;
    n.id = arr_of<20>(id, "id");
    n.addr = net::Addr::parse(addr, 0);
    return pyb(dht::encode_compact_node(n));
  });
  py::class_<dht::RoutingTable>(md, "RoutingTable")
      .def(py::init([](py::bytes own) { return new dht::RoutingTable(arr_of<20>(own, "id")); }))
      .def("insert", [](dht::RoutingTable& t, py::bytes id, std::string addr) {
        return t.insert({arr_of<20>(id, "id"), net::Addr::parse(addr, 0)});
      })
      .def("remove", [](dht::RoutingTable& t, py::bytes id) { t.remove(arr_of<20>(id, "id")); })
      .def("closest", [](const dht::RoutingTable& t, py::bytes target, size_t k) {
        py::list out;
        for (auto& n : t.closest(arr_of<20>(target, "target"), k)) out.append(py::make_tuple(pyb(n.id.data(), 20), n.addr.str()));
        return out;
      }, py::arg("target"), py::arg("k") = size_t(dht::K))
      .def("__len__", &dht::RoutingTable::size);
  py::class_<dht::Dht>(md, "Node")
      .def(py::init([](uint16_t port) {
             auto* d = new dht::Dht(port);
             d->start();
             return d;
           }), py::arg("port") = 0)
      .def_property_readonly("port", &dht::Dht::port)
      .def_property_readonly("id", [](const dht::Dht& d) { return pyb(d.id().data(), 20); })
      .def("bootstrap", [](dht::Dht& d, std::vector<std::string> nodes, int timeout_ms) {
        std::vector<net::Addr> a;
        for (auto& s : nodes) a.push_back(net::Addr::parse(s, 6881));
        py::gil_scoped_release nogil;
        return d.bootstrap(a, timeout_ms);
      }, py::arg("nodes"), py::arg("timeout_ms") = 2000)
      .def("get_peers", [](dht::Dht& d, py::bytes ih, int timeout_ms) {
        auto h = arr_of<20>(ih, "info_hash");
        std::vector<net::Addr> r;
        {
          py::gil_scoped_release nogil;
          r = d.get_peers(h, timeout_ms);
        }
        return addr_strs(r);
      }, py::arg("info_hash"), py::arg("timeout_ms") = 3000)
      .def("announce_peer", [](dht::Dht& d, py::bytes ih, uint16_t port, int timeout_ms) {
        auto h = arr_of<20>(ih, "info_hash");
        py::gil_scoped_release nogil;
        return d.announce_peer(h, port, timeout_ms);
      }, py::arg("info_hash"), py::arg("port"), py::arg("timeout_ms") = 3000)
      .def("ping", [](dht::Dht& d, std::string addr, int timeout_ms) {
        auto a = net::Addr::parse(addr, 6881);
        py::gil_scoped_release nogil;
        return d.ping(a, timeout_ms);
      }, py::arg("addr"), py::arg("timeout_ms") = 1000)
      .def("routing_size", [](dht::Dht& d) { return d.table().size(); })
      .def("stored_peers", [](const dht::Dht& d, py::bytes ih) { return addr_strs(d.stored_peers(arr_of<20>(ih, "info_hash"))); })
      .def("stats", [](const dht::Dht& d) {
        auto s = d.stats();
        py::dict r;
        r["queries_sent"] = s.queries_sent;
        r["responses"] = s.responses;
        r["queries_answered"] = s.queries_answered;
        r["timeouts"] = s.timeouts;
        r["lookups"] = s.lookups;
        return r;
      })
      .def("stop", [](dht::Dht& d) {
        py::gil_scoped_release nogil;
        d.stop();
      });

  // ---------------- small helpers (HTTP / hub) ----------------
  m.def("percent_encode", [](py::bytes b) {
    std::string s = b;
    return http::percent_encode(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  m.def("percent_decode", [](std::string s) { return pyb(http::percent_decode(s)); });
  m.def("extract_json_sha", [](std::string s) { return hub::extract_json_sha(s); });
  m.def("parse_reconstruction", [](std::string s) { return cas::reconstruction_to_json(cas::parse_reconstruction(s)); });

  // ---------------- config / cache ----------------
  m.def("config_json", []() { return Config::from_env().to_json(); });
  m.def("repo_folder_name", &repo_folder_name, py::arg("repo_id"), py::arg("type") = "model");
  m.def("list_cached_xorbs", []() { return storage::list_cached_xorbs(Config::from_env()); });
  m.def("cache_put_xorb", [](std::string hex, py::bytes data, int64_t range_start) {
    Config cfg = Config::from_env();
    storage::XorbCache c(cfg);
    std::string d = data;
    if (range_start < 0) c.put(hex, reinterpret_cast<const uint8_t*>(d.data()), d.size());
    else c.put_partial(hex, uint32_t(range_start), reinterpret_cast<const uint8_t*>(d.data()), d.size());
  }, py::arg("hex"), py::arg("data"), py::arg("range_start") = -1);
  m.def("cache_put_runs", [](std::vector<std::string> hexes, std::vector<uint32_t> offsets, std::vector<uintptr_t> ptrs,
                             std::vector<uint64_t> lens, int threads) {
    // Bulk cache fill straight from memory (e.g. a pinned origin): run i = chunks from offset[i] on.
    if (offsets.size() != hexes.size() || ptrs.size() != hexes.size() || lens.size() != hexes.size())
      throw std::invalid_argument("cache_put_runs: lists of different lengths");
    Config cfg = Config::from_env();
    storage::XorbRegistry reg;
    storage::XorbCache c(cfg, &reg);
    py::gil_scoped_release nogil;
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < hexes.size();)
        c.put_run(hexes[i], offsets[i], reinterpret_cast<const uint8_t*>(ptrs[i]), lens[i], true);
    };
    std::vector<std::thread> ts;
    for (int t = 1; t < std::max(1, threads); ++t) ts.emplace_back(work);
    work();
    for (auto& t : ts) t.join();
    return hexes.size();
  }, py::arg("hexes"), py::arg("offsets"), py::arg("ptrs"), py::arg("lens"), py::arg("threads") = 8);

  // ---------------- BT seeder / peer client ----------------
  py::class_<PySeeder>(m, "Seeder", "BT listener serving the local xorb cache over ut_xet")
      .def(py::init<int, std::string>(), py::arg("port") = 0, py::arg("fault") = "")
      .def_property_readonly("port", [](const PySeeder& s) { return s.server->port(); })
      .def("rescan", [](PySeeder& s) { s.registry.scan(s.cfg); })
      .def("stats", [](const PySeeder& s) {
        auto st = s.server->stats();
        py::dict r;
        r["active_peers"] = st.active_peers;
        r["total_peers"] = st.total_peers;
        r["chunks_served"] = st.chunks_served;
        r["bytes_served"] = st.bytes_served;
        r["not_found"] = st.not_found;
        r["rejected"] = st.rejected;
        return r;
      })
      .def("stop", [](PySeeder& s) {
        py::gil_scoped_release nogil;
        s.server->stop();
      });
  m.def("peer_fetch", [](std::string addr, py::bytes xorb_hash, uint32_t start, uint32_t end, int timeout_ms) {
    auto h = arr_of<32>(xorb_hash, "xorb hash");
    auto a = net::Addr::parse(addr, 6881);
    bt::ChunkResult r;
    std::string client;
    {
      py::gil_scoped_release nogil;
      auto me = peer_id::generate();
      auto sess = bt::PeerSession::connect(a, peer_id::info_hash(h.data()), me, 0, timeout_ms);
      if (!sess->supports_xet()) throw Error("PeerNoXet", addr);
      bt::XetRequest req;
      req.xorb_hash = h;
      req.range_start = start;
      req.range_end = end;
      r = sess->request(req, timeout_ms);
      client = sess->client();
    }
    return py::make_tuple(pyb(r.data), r.chunk_offset, client);
  }, py::arg("addr"), py::arg("xorb_hash"), py::arg("start"), py::arg("end"), py::arg("timeout_ms") = 5000);

  // Persistent BEP XET client connection (pipelined requests; any xorb over one connection).
  py::class_<bt::PeerSession, std::shared_ptr<bt::PeerSession>>(m, "PeerConnection")
      .def(py::init([](std::string addr, py::bytes first_xorb, int timeout_ms) {
             auto a = net::Addr::parse(addr, 6881);
             auto h = arr_of<32>(first_xorb, "xorb hash");
             py::gil_scoped_release nogil;
             return bt::PeerSession::connect(a, peer_id::info_hash(h.data()), peer_id::generate(), 0, timeout_ms);
           }),
           py::arg("addr"), py::arg("xorb_hash"), py::arg("timeout_ms") = 5000)
      .def_property_readonly("supports_xet", &bt::PeerSession::supports_xet)
      .def_property_readonly("client", &bt::PeerSession::client)
      .def("fetch", [](bt::PeerSession& s, py::bytes xorb_hash, uint32_t a, uint32_t b, int timeout_ms) {
        bt::XetRequest r;
        r.xorb_hash = arr_of<32>(xorb_hash, "xorb hash");
        r.range_start = a;
        r.range_end = b;
        bt::ChunkResult res;
        {
          py::gil_scoped_release nogil;
          res = s.request(r, timeout_ms);
        }
        return py::make_tuple(pyb(res.data), res.chunk_offset);
      }, py::arg("xorb_hash"), py::arg("start"), py::arg("end"), py::arg("timeout_ms") = 30000)
      .def("fetch_many_bytes", [](bt::PeerSession& s, std::vector<py::bytes> hashes, std::vector<uint32_t> starts,
                                  std::vector<uint32_t> ends, int timeout_ms) {
        // Pipelined; returns total payload bytes (the data is discarded: for load generation).
        // Load generation: every payload is received into one reused per-thread buffer (like iperf's
        // receiver), so the client does not pay a fresh 64 MiB allocation's page faults per response.
        thread_local std::vector<uint8_t> scratch;
        auto sink = [](size_t n) -> uint8_t* {
          if (scratch.size() < n) scratch.resize(n);
          return scratch.data();
        };
        std::vector<bt::XetRequest> reqs(hashes.size());
        for (size_t i = 0; i < hashes.size(); ++i) {
          reqs[i].xorb_hash = arr_of<32>(hashes[i], "xorb hash");
          reqs[i].range_start = starts.at(i);
          reqs[i].range_end = ends.at(i);
          reqs[i].sink = sink;
        }
        uint64_t total = 0;
        size_t failed = 0;
        {
          py::gil_scoped_release nogil;
          std::vector<std::string> errs;
          auto res = s.request_many(reqs, timeout_ms, &errs);
          for (size_t i = 0; i < res.size(); ++i) {
            total += res[i].ext ? res[i].ext_len : res[i].data.size();
            if (i < errs.size() && !errs[i].empty()) failed++;
          }
        }
        return py::make_tuple(total, failed);
      }, py::arg("hashes"), py::arg("starts"), py::arg("ends"), py::arg("timeout_ms") = 60000);

  // ---------------- in-memory Xet fetch (host waterfall, no snapshot) ----------------
  // The host twin of _hip.DeviceXetPull: Xet files reconstructed through the cache -> P2P -> CDN
  // waterfall and verified against their file hash, written into caller memory (e.g. a CPU tensor)
  // instead of the HF cache.  Kept alive across calls so peer connections and the CAS session carry
  // over (swarm_pull rounds on CPU process groups).
  py::class_<HostXetFetcher>(m, "HostXetFetcher")
      .def(py::init([](const std::string& repo, const std::string& revision, const std::string& repo_type, bool p2p,
                       std::vector<std::string> peers, std::optional<std::string> tracker, bool dht,
                       std::vector<std::string> boot, int concurrency) {
             py::gil_scoped_release nogil;
             return new HostXetFetcher(repo, revision, repo_type, p2p, std::move(peers), std::move(tracker), dht,
                                       std::move(boot), concurrency);
           }),
           py::arg("repo"), py::arg("revision") = "main", py::arg("repo_type") = "model", py::arg("p2p") = true,
           py::arg("peers") = std::vector<std::string>{}, py::arg("tracker") = std::nullopt, py::arg("dht") = true,
           py::arg("dht_bootstrap") = std::vector<std::string>{}, py::arg("concurrency") = 0)
      .def("fetch_files",
           [](HostXetFetcher& self, const std::vector<std::tuple<std::string, uintptr_t, uint64_t>>& files) {
             std::vector<FileResult> rs;
             {
               py::gil_scoped_release nogil;
               rs = self.fetch(files);
             }
             py::list out;
             for (auto& r : rs) {
               py::dict d;
               d["bytes"] = r.bytes;
               d["terms"] = r.terms;
               d["seconds"] = r.seconds;
               d["chunk_lens"] = py::bytes(reinterpret_cast<const char*>(r.chunk_lens.data()), 4 * r.chunk_lens.size());
               out.append(d);
             }
             return out;
           },
           py::arg("files"), "[(xet_hash, ptr, size), ...] -> one dict per file (chunk_lens: uint32 sizes)")
      .def("term_shapes", [](HostXetFetcher& self, const std::string& hex) {
             std::vector<TermShape> v;
             {
               py::gil_scoped_release nogil;
               v = self.shapes(hex);
             }
             return term_shapes_py(v);
           }, py::arg("xet_hash"), "[(unpacked_length, n_chunks), ...] of the file's reconstruction terms")
      .def("term_keys", [](HostXetFetcher& self, const std::string& hex) {
             std::vector<zest::TermKey> v;
             {
               py::gil_scoped_release nogil;
               v = self.term_keys(hex);
             }
             return zest::term_keys_py(v);
           }, py::arg("xet_hash"), "[(xorb_hex, chunk_start, chunk_end), ...] of the file's reconstruction terms")
      .def("cached_terms", [](HostXetFetcher& self, std::vector<std::string> hexes, std::vector<uint32_t> starts,
                              std::vector<uint32_t> ends) {
             std::vector<uint8_t> v;
             {
               py::gil_scoped_release nogil;
               v = self.cached_terms(hexes, starts, ends);
             }
             return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
           }, py::arg("hexes"), py::arg("starts"), py::arg("ends"),
           "one byte per term: 1 when the local xorb cache covers its chunk range (planner possession check)")
      .def("reset_reconstructions", &HostXetFetcher::reset_reconstructions, "forget cached reconstructions (between pulls)")
      .def("fetch_terms",
           [](HostXetFetcher& self, const std::vector<std::tuple<std::string, uint32_t, uint32_t, uintptr_t, uint64_t>>& v,
              uintptr_t hashes, bool repair) {
             const auto jobs = term_jobs_of(v);
             std::vector<TermJobResult> rs;
             {
               py::gil_scoped_release nogil;
               rs = self.fetch_terms(jobs, reinterpret_cast<uint8_t*>(hashes), repair);
             }
             return term_results_py(rs);
           },
           py::arg("jobs"), py::arg("hashes_ptr"), py::arg("repair") = false,
           "[(xet_hash, t0, t1, dst_ptr, chunk0), ...]: fetch + decode + chunk-hash term ranges into host memory")
      .def("settle", [](HostXetFetcher& self, const std::string& hex, bool ok) {
             py::gil_scoped_release nogil;
             return self.settle(hex, ok);
           }, py::arg("xet_hash"), py::arg("ok"), "publish (ok) or drop the file's quarantined runs")
      .def("stats_json", &HostXetFetcher::stats_json);

  // ---------------- pull ----------------
  m.def("pull", [](std::string repo, std::string revision, bool p2p, std::vector<std::string> peers,
                   std::optional<std::string> tracker_url, bool dht, std::vector<std::string> dht_bootstrap,
                   std::vector<std::string> include, bool verify, int concurrency, std::string repo_type) {
    Config cfg = Config::from_env();
    PullOptions o;
    o.repo_id = repo;
    o.revision = revision;
    o.p2p = p2p;
    o.peers = peers;
    o.tracker = tracker_url;
    o.dht = dht;
    o.dht_bootstrap = dht_bootstrap;
    o.include = include;
    o.verify = verify;
    o.concurrency = concurrency;
    o.repo_type = repo_type;
    o.autostart_server = false;
    std::ostringstream out, err;
    PullSummary s;
    {
      py::gil_scoped_release nogil;
      s = run_pull(cfg, o, out, err);
    }
    py::dict d;
    d["snapshot_dir"] = s.snapshot_dir;
    d["commit"] = s.commit;
    d["bytes"] = s.bytes;
    d["files"] = s.files;
    d["xet_files"] = s.xet_files;
    d["cached_files"] = s.cached_files;
    d["bytes_from_peer"] = s.bytes_from_peer;
    d["bytes_from_cdn"] = s.bytes_from_cdn;
    d["bytes_from_cache"] = s.bytes_from_cache;
    d["seconds"] = s.seconds;
    d["stats_json"] = s.stats_json;
    d["files_json"] = s.files_json;
    d["failed_files"] = s.failed_files;
    d["stdout"] = out.str();
    d["stderr"] = err.str();
    return d;
  }, py::arg("repo"), py::arg("revision") = "main", py::arg("p2p") = true, py::arg("peers") = std::vector<std::string>{},
     py::arg("tracker") = std::nullopt, py::arg("dht") = true, py::arg("dht_bootstrap") = std::vector<std::string>{},
     py::arg("include") = std::vector<std::string>{}, py::arg("verify") = true, py::arg("concurrency") = 0,
     py::arg("repo_type") = "model");
  m.def("write_ref", [](std::string repo, std::string ref, std::string commit, std::string repo_type) {
    Config cfg = Config::from_env();
    (void)repo_type;
    storage::write_ref(cfg, repo, ref, commit);
  }, py::arg("repo"), py::arg("ref"), py::arg("commit"), py::arg("repo_type") = "model");
  m.def("write_verified_marker", [](std::string repo, std::string commit, std::string path, std::string xet_hex,
                                    std::string file) {
    Config cfg = Config::from_env();
    storage::write_verified_marker(cfg, repo, commit, path, xet_hex, file);
  }, py::arg("repo"), py::arg("commit"), py::arg("path"), py::arg("xet_hash"), py::arg("file"),
     "Record that `file` (snapshot path) was verified against its Xet hash");
  m.def("check_verified_marker", [](std::string repo, std::string commit, std::string path, std::string xet_hex,
                                    std::string file) {
    Config cfg = Config::from_env();
    return storage::check_verified_marker(cfg, repo, commit, path, xet_hex, file);
  }, py::arg("repo"), py::arg("commit"), py::arg("path"), py::arg("xet_hash"), py::arg("file"),
     "True when `file` carries a verified marker matching its Xet hash, size and mtime");
  m.def("xet_hash_of_file", [](std::string file, int threads) {
    py::gil_scoped_release nogil;
    return storage::xet_hash_of_file(file, threads);
  }, py::arg("file"), py::arg("threads") = 0, "Xet file hash of a file on disk (CDC + BLAKE3 + Merkle)");
  // ---------------- in-process memory origin (mem:// fetch_info URLs; hub.h) ----------------
  m.def("mem_origin_add", [](std::vector<std::string> hexes, std::vector<uint64_t> starts, std::vector<uintptr_t> ptrs,
                             std::vector<uint64_t> lens) {
    if (starts.size() != hexes.size() || ptrs.size() != hexes.size() || lens.size() != hexes.size())
      throw std::invalid_argument("mem_origin_add: lists of different lengths");
    for (size_t i = 0; i < hexes.size(); ++i)
      cas::mem_origin_add(hexes[i], starts[i], reinterpret_cast<const uint8_t*>(ptrs[i]), lens[i]);
    return cas::mem_origin_size();
  }, py::arg("xorb_hexes"), py::arg("url_starts"), py::arg("ptrs"), py::arg("lens"),
     "serve fetch_info url_range [start, start + len) of each xorb from host memory at ptr (caller keeps it alive)");
  m.def("mem_origin_clear", &cas::mem_origin_clear);
  m.def("mem_origin_size", &cas::mem_origin_size);

  m.def("list_repo_files", [](std::string repo, std::string revision, std::string repo_type) {
    Config cfg = Config::from_env();
    std::vector<hub::RepoFile> files;
    std::optional<std::string> sha;
    {
      py::gil_scoped_release nogil;
      files = hub::list_files(cfg, repo, revision, repo_type);
      sha = hub::resolve_commit(cfg, repo, revision, repo_type);
    }
    py::list out;
    for (auto& f : files) {
      py::dict d;
      d["path"] = f.path;
      d["size"] = f.size;
      d["xet_hash"] = f.xet_hash ? py::object(py::str(*f.xet_hash)) : py::object(py::none());
      out.append(d);
    }
    return py::make_tuple(sha ? py::object(py::str(*sha)) : py::object(py::none()), out);
  }, py::arg("repo"), py::arg("revision") = "main", py::arg("repo_type") = "model");
  m.def("server_healthy", &server_healthy, py::arg("http_port"), py::arg("timeout_ms") = 1000);

  // ---------------- tracing (shared with the C++ spans) ----------------
  auto mtr = m.def_submodule("trace", "host tracing: ZEST_TRACE=1 (log) or ZEST_TRACE=file.json (Chrome trace)");
  mtr.def("enabled", &trace::enabled);
  mtr.def("mode", &trace::mode);
  mtr.def("now_us", &trace::now_us);
  mtr.def("roctx_enabled", &trace::roctx_enabled);
  mtr.def("roctx_push", &trace::roctx_push);
  mtr.def("roctx_pop", &trace::roctx_pop);
  mtr.def("log", [](const std::string& cat, const std::string& msg) { trace::log(cat.c_str(), msg); });
  mtr.def("complete", [](const std::string& cat, const std::string& name, uint64_t ts, uint64_t dur,
                         const std::string& args) {
    // cat must outlive the call only; complete() copies it into the event string
    trace::complete(cat.c_str(), name, ts, dur, args);
  }, py::arg("cat"), py::arg("name"), py::arg("ts_us"), py::arg("dur_us"), py::arg("args_json") = "");
  mtr.def("counter", &trace::counter);
  mtr.def("flush", &trace::flush);
  mtr.def("set_output", &trace::set_output);

  // ---------------- synthetic bench ----------------
  m.def("bench_synthetic", [](bool extended) {
    std::vector<bench::Result> r;
    {
      py::gil_scoped_release nogil;
      r = bench::run_synthetic(extended);
    }
    py::list out;
    for (auto& x : r) {
      py::dict d;
      d["name"] = x.name;
      d["runs"] = x.runs;
      d["median_ns"] = x.median_ns;
      d["throughput_mbps"] = x.throughput_mbps();
      d["bytes_processed"] = x.bytes_processed;
      out.append(d);
    }
    return out;
  }, py::arg("extended") = true);
}
