// Native unit tests of the host core (no Python): codecs, Xet formats, protocol framing, storage.
// Built by `python tools/build.py --only tests` (and `--asan` for an ASan/UBSan build) or CMake
// (`ctest`), run by tests/test_cpp_core.py.  Vectors are independent of the reference's Zig tests
// (port the assertions, not the code).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "bencode.h"
#include "blake3.h"
#include "bt_peer.h"
#include "bt_server.h"
#include "bt_wire.h"
#include "cdc.h"
#include "config.h"
#include "dht.h"
#include "http.h"
#include "json.h"
#include "lz4.h"
#include "sha1.h"
#include "storage.h"
#include "term_jobs.h"
#include "tracker.h"
#include "xet_hash.h"
#include "xorb.h"

using namespace zest;

namespace {

int g_failed = 0, g_checks = 0;
std::vector<std::pair<const char*, std::function<void()>>>& registry() {
  static std::vector<std::pair<const char*, std::function<void()>>> r;
  return r;
}
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().emplace_back(n, std::move(f)); }
};
#define TEST(name)                         \
  static void name();                      \
  static Reg reg_##name(#name, name);      \
  static void name()
#define CHECK(c)                                                               \
  do {                                                                         \
    ++g_checks;                                                                \
    if (!(c)) {                                                                \
      ++g_failed;                                                              \
      std::fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
    }                                                                          \
  } while (0)
#define CHECK_THROWS(expr, want)                 \
  do {                                           \
    bool thrown = false;                         \
    try {                                        \
      expr;                                      \
    } catch (const Error& e) {                   \
      thrown = e.code() == (want);               \
    }                                            \
    CHECK(thrown);                               \
  } while (0)

std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

Bytes rnd(size_t n, uint32_t seed, int alphabet = 256) {
  std::mt19937 g(seed);
  Bytes b(n);
  for (auto& x : b) x = uint8_t(g() % unsigned(alphabet));
  return b;
}

}  // namespace

TEST(blake3_vectors) {
  uint8_t out[32];
  blake3::hash("", 0, out);
  CHECK(hex(out, 32) == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262");
  blake3::hash("abc", 3, out);
  CHECK(hex(out, 32) == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85");
  // all SIMD backends agree on a multi-chunk message
  Bytes big = rnd(1 << 20, 7);
  uint8_t ref[32];
  blake3::force_backend("portable");
  blake3::hash(big.data(), big.size(), ref);
  for (const char* be : {"avx2", "avx512"}) {
    if (!blake3::force_backend(be)) continue;
    blake3::hash(big.data(), big.size(), out);
    CHECK(std::memcmp(out, ref, 32) == 0);
  }
  blake3::force_backend("auto");
}

TEST(sha1_vectors) {
  auto d = Sha1::hash("abc", 3);
  CHECK(hex(d.data(), 20) == "a9993e364706816aba3e25717850c26c9cd0d89d");
  auto e = Sha1::hash("", 0);
  CHECK(hex(e.data(), 20) == "da39a3ee5e6b4b0d3255bfef95601890afd80709");
  uint8_t h[32];
  std::memset(h, 0xAB, 32);
  std::string msg = "zest-xet-v1:" + std::string(reinterpret_cast<char*>(h), 32);
  CHECK(peer_id::info_hash(h) == Sha1::hash(msg.data(), msg.size()));
  auto pid = peer_id::generate();
  CHECK(std::memcmp(pid.data(), peer_id::kClientPrefix, 8) == 0);
}

TEST(bencode_codec) {
  bencode::Document doc;
  auto r = bencode::decode(doc, "d1:md6:ut_xeti1ee1:pi6881e1:v8:zest/0.4e");
  CHECK(r.is_dict() && r.get("m").get_int("ut_xet", 0) == 1 && r.get_int("p", 0) == 6881);
  CHECK(r.get_str("v") == "zest/0.4");
  CHECK(bencode::encode(r) == "d1:md6:ut_xeti1ee1:pi6881e1:v8:zest/0.4e");
  CHECK_THROWS(bencode::decode(doc, "i03e"), "LeadingZero");
  CHECK_THROWS(bencode::decode(doc, "i-0e"), "NegativeZero");
  CHECK_THROWS(bencode::decode(doc, "d1:b0:1:a0:e"), "UnsortedDictKeys");
  CHECK_THROWS(bencode::decode(doc, "l"), "UnexpectedEnd");
  std::string deep(100, 'l');
  deep += std::string(100, 'e');
  bool threw = false;
  try {
    bencode::decode(doc, deep);
  } catch (const Error&) {
    threw = true;
  }
  CHECK(threw);
}

TEST(bt_wire_and_bep_xet) {
  Sha1Digest ih{};
  ih.fill(7);
  auto pid = peer_id::generate();
  Bytes hs;
  bt::write_handshake(hs, ih, pid);
  CHECK(hs.size() == 68);
  auto h = bt::parse_handshake(hs.data());
  CHECK(h.info_hash == ih && h.peer_id == pid && h.supports_bep10());
  Bytes m;
  uint8_t pl[3] = {1, 2, 3};
  bt::write_message(m, bt::kRequest, pl, 3);
  bt::Message msg;
  CHECK(bt::parse_message(m.data(), m.size(), msg) == m.size() && msg.id == bt::kRequest && msg.payload.size == 3);
  CHECK(bt::parse_message(m.data(), 3, msg) == 0);
  uint8_t xh[32];
  for (int i = 0; i < 32; ++i) xh[i] = uint8_t(i);
  Bytes rq;
  bep_xet::encode_chunk_request(rq, 3, 99, xh, 2, 5);
  CHECK(rq.size() == 51);
  auto x = bep_xet::decode(ByteSpan(rq.data() + 6, rq.size() - 6));
  CHECK(x.type == bep_xet::kChunkRequest && x.request_id == 99 && x.range_start == 2 && x.range_end == 5);
  auto caps = bep_xet::parse_ext_handshake(ByteSpan(bep_xet::make_ext_handshake(1234, 9)));
  CHECK(caps.ut_xet_id == 9 && caps.listen_port == 1234);
}

TEST(lz4_and_bg4) {
  for (uint32_t seed = 0; seed < 6; ++seed) {
    for (size_t n : {size_t(0), size_t(1), size_t(100), size_t(65536), size_t(70000), size_t(131072)}) {
      Bytes src = rnd(n, seed, seed % 2 ? 4 : 256);
      Bytes fr = lz4::compress_frame(src.data(), src.size());
      Bytes back = lz4::decompress_frame(fr.data(), fr.size(), src.size());
      CHECK(back == src);
      Bytes g(n), u(n);
      bg4::split(src.data(), n, g.data());
      bg4::join(g.data(), n, u.data());
      CHECK(u == src);
    }
  }
  Bytes junk = rnd(64, 3);
  bool threw = false;
  try {
    lz4::decompress_frame(junk.data(), junk.size(), 100);
  } catch (const Error&) {
    threw = true;
  }
  CHECK(threw);
}

TEST(xorb_roundtrip_and_footer) {
  for (auto pol : {xet::CompressionPolicy::None, xet::CompressionPolicy::LZ4, xet::CompressionPolicy::BG4,
                   xet::CompressionPolicy::Auto}) {
    xet::XorbBuilder b(pol);
    std::vector<Bytes> chunks;
    for (uint32_t i = 0; i < 5; ++i) {
      chunks.push_back(rnd(9000 + 1000 * i, i, i % 2 ? 3 : 256));
      b.add_chunk(chunks.back().data(), chunks.back().size());
    }
    Bytes blob = b.serialize(true);
    auto idx = xet::index_chunks(blob.data(), blob.size());
    CHECK(idx.size() == 5);
    auto f = xet::parse_footer(blob.data(), blob.size());
    CHECK(f.has_value() && f->xorb_hash == b.hash() && f->chunk_hashes.size() == 5);
    Bytes out;
    std::vector<xet::HashSize> hs;
    xet::extract_chunk_range(blob.data(), blob.size(), 1, 4, out, &hs);
    Bytes want;
    for (int i = 1; i < 4; ++i) want.insert(want.end(), chunks[i].begin(), chunks[i].end());
    CHECK(out == want && hs.size() == 3 && hs[0].hash == xet::chunk_hash(chunks[1].data(), chunks[1].size()));
  }
}

TEST(cdc_constraints) {
  Bytes data = rnd(8 << 20, 11);
  auto ends = xet::chunk_ends(data.data(), data.size());
  uint64_t prev = 0;
  bool ok = !ends.empty() && ends.back() == data.size();
  for (size_t i = 0; i < ends.size(); ++i) {
    const uint64_t len = ends[i] - prev;
    if (len > 131072 || (len < 8192 && i + 1 != ends.size())) ok = false;
    prev = ends[i];
  }
  CHECK(ok);
  // shift invariance: boundaries after an inserted prefix re-synchronise
  Bytes shifted(1000, 0x55);
  shifted.insert(shifted.end(), data.begin(), data.end());
  auto e2 = xet::chunk_ends(shifted.data(), shifted.size());
  size_t common = 0;
  for (auto e : e2)
    for (auto f : ends)
      if (e == f + 1000) ++common;
  CHECK(common > ends.size() / 2);
}

TEST(merkle_rules) {
  std::vector<xet::HashSize> leaves;
  for (uint32_t i = 0; i < 100; ++i) {
    Bytes c = rnd(100, i);
    leaves.push_back({xet::chunk_hash(c.data(), c.size()), 100});
  }
  // a group closes after at most 9 children and never before 2 (except the tail)
  size_t p = 0;
  while (p < leaves.size()) {
    const size_t cut = xet::next_merge_cut(leaves.data() + p, leaves.size() - p);
    CHECK(cut >= 1 && cut <= 9 && (cut >= 2 || leaves.size() - p < 2));
    p += cut;
  }
  auto root = xet::merkle_root(leaves);
  CHECK(xet::file_hash(leaves) == xet::file_hash_from_root(root, false));
  CHECK(xet::from_hex(xet::to_hex(root)) == root);
}

TEST(json_and_http_helpers) {
  auto v = json::Value::parse(R"({"a":[1,2,{"b":"x\"y"}],"n":-3.5,"t":true,"z":null})");
  CHECK(v["a"].size() == 3 && v["a"].at(2).str_or("b", "") == "x\"y" && v["t"].as_bool() && v["z"].is_null());
  json::Writer w;
  w.obj().key("k").str("v\n").key("n").num(int64_t(5)).end();
  CHECK(json::Value::parse(w.out()).str_or("k", "") == "v\n");
  auto u = http::Url::parse("https://example.com:8443/a/b?x=1");
  CHECK(u.scheme == "https" && u.host == "example.com" && u.port == 8443 && u.target == "/a/b?x=1");
  auto u2 = http::Url::parse("http://h/");
  CHECK(u2.port == 80);
  uint8_t raw[3] = {0, 0x41, 0xff};
  CHECK(http::percent_encode(raw, 3) == "%00A%FF");
  CHECK(http::percent_decode("%00A%FF") == std::string("\0A\xff", 3));
}

TEST(dht_routing) {
  dht::NodeId own{};
  dht::RoutingTable t(own);
  for (int i = 0; i < 40; ++i) {
    dht::NodeId id{};
    id[19] = uint8_t(i + 1);
    id[0] = uint8_t(i * 6);
    t.insert({id, net::Addr::parse("127.0.0.1:" + std::to_string(2000 + i), 0)});
  }
  dht::NodeId target{};
  auto c = t.closest(target, 8);
  CHECK(c.size() == 8);
  for (size_t i = 1; i < c.size(); ++i) CHECK(!dht::closer(target, c[i].id, c[i - 1].id));
  auto compact = dht::encode_compact_node(c[0]);
  auto back = dht::parse_compact_nodes(compact);
  CHECK(back.size() == 1 && back[0].id == c[0].id && back[0].addr == c[0].addr);
  auto peers = tracker::parse_compact_peers(std::string("\x0a\x00\x00\x05\x1a\xe1", 6));
  CHECK(peers.size() == 1 && peers[0].str() == "10.0.0.5:6881");
}

TEST(xorb_cache_runs) {
  char tmpl[] = "/tmp/zest_cpp_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  setenv("ZEST_CACHE_DIR", dir, 1);
  Config cfg = Config::from_env();
  storage::XorbCache cache(cfg);
  xet::XorbBuilder b(xet::CompressionPolicy::None);
  for (uint32_t i = 0; i < 6; ++i) {
    Bytes c = rnd(9000, i);
    b.add_chunk(c.data(), c.size());
  }
  const std::string hx = xet::to_hex(b.hash());
  Bytes body = b.body();
  auto idx = xet::index_chunks(body.data(), body.size());
  // cache a prefix run [0,2) under the "full" name and a partial run [3,6)
  const uint64_t p2 = idx[2].header_off;
  cache.put_run(hx, 0, body.data(), p2);
  cache.put_run(hx, 3, body.data() + idx[3].header_off, body.size() - idx[3].header_off);
  CHECK(cache.find(hx, 0, 2).has_value());
  CHECK(!cache.find(hx, 0, 3).has_value());  // the prefix must not be served as the whole xorb
  auto h = cache.find(hx, 4, 6);
  CHECK(h.has_value() && h->chunk_offset == 4 && xet::index_chunks(h->bytes(), h->size()).size() == 2);
  // zero-copy view of the file mapping, equal to the original bytes of chunks [4, 6)
  CHECK(h.has_value() && h->size() == body.size() - idx[4].header_off &&
        std::memcmp(h->bytes(), body.data() + idx[4].header_off, h->size()) == 0);
  h->materialize();
  CHECK(h->data.size() == body.size() - idx[4].header_off);
  CHECK(!cache.find(hx, 2, 4).has_value());
  CHECK(storage::list_cached_xorbs(cfg).size() == 1);
}

TEST(xorb_cache_covers_and_write_behind) {
  // covers(): the planner's header-only possession check agrees with find(); the write-behind
  // writer keeps per-xorb order (a promote queued after its quarantine write publishes it), drops
  // runs over its byte bound instead of blocking, and flush() waits for everything queued.
  char tmpl[] = "/tmp/zest_cpp_wb_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  setenv("ZEST_CACHE_DIR", dir, 1);
  Config cfg = Config::from_env();
  storage::XorbRegistry reg;
  storage::XorbCache cache(cfg, &reg);
  xet::XorbBuilder b(xet::CompressionPolicy::None);
  for (uint32_t i = 0; i < 5; ++i) {
    Bytes c = rnd(9000, 70 + i);
    b.add_chunk(c.data(), c.size());
  }
  const std::string hx = xet::to_hex(b.hash());
  Bytes body = b.body();
  auto idx = xet::index_chunks(body.data(), body.size());
  CHECK(!cache.covers(hx, 0, 1));
  {
    storage::CacheWriter w(&cache, 1 << 20, 2);
    CHECK(w.put_run(hx, 2, body.data() + idx[2].header_off, body.size() - idx[2].header_off, false));
    const std::string pend = w.put_pending(hx, 0, body.data(), idx[2].header_off);
    CHECK(!pend.empty());
    w.promote(hx, 0, pend);
    Bytes big(2 << 20, 7);
    CHECK(!w.put_run(hx, 9, big.data(), big.size(), false));  // over the bound: dropped, not queued
    w.flush();
    auto st = w.stats();
    CHECK(st.dropped_bytes == big.size() && st.written_bytes == body.size());
    CHECK(!storage::exists(pend));  // promoted (renamed) after its own write
  }
  CHECK(cache.covers(hx, 0, 2) && cache.find(hx, 0, 2).has_value());
  CHECK(cache.covers(hx, 3, 5) && cache.find(hx, 3, 5).has_value());
  CHECK(!cache.covers(hx, 1, 3) && !cache.find(hx, 1, 3).has_value());  // no run spans chunks 1..2
  CHECK(!cache.covers(hx, 2, 6));
  auto held = cached_terms(cache, {hx, hx, hx}, {0, 1, 2}, {2, 3, 5}, 2);
  CHECK(held == std::vector<uint8_t>({1, 0, 1}));
}

TEST(xorb_cache_write_behind_ref_copies_and_registry_lookup) {
  // put_pending_ref / put_run_ref: the caller's bytes are copied by the writer's copy threads;
  // on_copied runs exactly once per queued run (never for a dropped one), the written runs equal the
  // caller's bytes even though the caller overwrites its buffer right after on_copied, and a promote
  // queued after on_copied publishes the run.  registry lookup: find() of an unregistered xorb
  // answers from the registry, a run published through the writer is found.
  char tmpl[] = "/tmp/zest_cpp_wbref_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  setenv("ZEST_CACHE_DIR", dir, 1);
  Config cfg = Config::from_env();
  storage::XorbRegistry reg;
  reg.scan(cfg);
  storage::XorbCache cache(cfg, &reg);
  cache.set_registry_lookup(true);
  xet::XorbBuilder b(xet::CompressionPolicy::None);
  for (uint32_t i = 0; i < 6; ++i) {
    Bytes c = rnd(9000, 90 + i);
    b.add_chunk(c.data(), c.size());
  }
  const std::string hx = xet::to_hex(b.hash());
  const Bytes body = b.body();
  auto idx = xet::index_chunks(body.data(), body.size());
  CHECK(!cache.maybe_cached(hx) && !cache.find(hx, 0, 1).has_value());
  {
    storage::CacheWriter w(&cache, 1 << 20, 2);
    std::mutex mu;
    std::condition_variable cv;
    int copied = 0;
    auto done = [&] {
      std::lock_guard<std::mutex> g(mu);
      ++copied;
      cv.notify_all();
    };
    Bytes buf1(body.begin(), body.begin() + long(idx[3].header_off));  // chunks 0..2, as a peer run
    const std::string pend = w.put_pending_ref(hx, 0, buf1.data(), buf1.size(), done);
    CHECK(!pend.empty());
    const size_t tail = body.size() - idx[3].header_off;
    Bytes buf2(body.begin() + long(idx[3].header_off), body.end());  // chunks 3..5, as a CDN run
    CHECK(w.put_run_ref(hx, 3, buf2.data(), tail, false, done));
    Bytes big(2 << 20, 7);
    CHECK(!w.put_run_ref(hx, 9, big.data(), big.size(), false, done));  // dropped: no callback
    {
      std::unique_lock<std::mutex> g(mu);
      CHECK(cv.wait_for(g, std::chrono::seconds(10), [&] { return copied == 2; }));
    }
    std::fill(buf1.begin(), buf1.end(), 0);  // the caller reuses its memory once copied
    std::fill(buf2.begin(), buf2.end(), 0);
    w.promote(hx, 0, pend);
    w.flush();
    CHECK(copied == 2 && w.stats().written_bytes == body.size());
  }
  CHECK(cache.maybe_cached(hx));
  auto h0 = cache.find(hx, 0, 3), h1 = cache.find(hx, 3, 6);
  CHECK(h0.has_value() && h1.has_value());
  CHECK(h0->size() == idx[3].header_off && std::memcmp(h0->bytes(), body.data(), h0->size()) == 0);
  CHECK(std::memcmp(h1->bytes(), body.data() + idx[3].header_off, h1->size()) == 0);
}

TEST(xorb_cache_quarantine_per_fetch) {
  // Two concurrent fetches of the same run (e.g. two files, two peers) quarantine under distinct
  // names; promote() publishes exactly the copy of the file that verified, discard() drops the
  // other; a quarantine file whose writer is gone is swept, a live one stays.
  char tmpl[] = "/tmp/zest_cpp_q_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  setenv("ZEST_CACHE_DIR", dir, 1);
  Config cfg = Config::from_env();
  storage::XorbCache cache(cfg);
  xet::XorbBuilder b(xet::CompressionPolicy::None);
  for (uint32_t i = 0; i < 3; ++i) {
    Bytes c = rnd(9000, 40 + i);
    b.add_chunk(c.data(), c.size());
  }
  const std::string hx = xet::to_hex(b.hash());
  Bytes good = b.body(), bad = good;
  bad[100] ^= 1;
  const std::string p_bad = cache.put_pending(hx, 0, bad.data(), bad.size());
  const std::string p_good = cache.put_pending(hx, 0, good.data(), good.size());
  CHECK(p_bad != p_good && storage::exists(p_bad) && storage::exists(p_good));
  CHECK(!cache.find(hx, 0, 3).has_value());  // quarantined runs are invisible
  CHECK(storage::list_cached_xorbs(cfg).empty());
  CHECK(cache.promote(hx, 0, p_good));
  cache.discard_pending(p_bad);
  auto h = cache.find(hx, 0, 3);
  CHECK(h.has_value() && h->size() == good.size() && std::memcmp(h->bytes(), good.data(), good.size()) == 0);
  CHECK(!storage::exists(p_bad) && !storage::exists(p_good));
  // stale sweep: a live writer's file stays, a dead writer's (pid that cannot exist) goes
  const std::string live = cache.put_pending(hx, 1, good.data(), good.size());
  const std::string dead = live.substr(0, live.rfind(".p")) + ".p999999999-0.unverified";
  storage::write_file_atomic(dead, good.data(), good.size(), false);
  CHECK(!storage::stale_pending(live, 3600) && storage::stale_pending(dead, 3600));
  CHECK(cache.sweep_pending(3600) == 1);
  CHECK(storage::exists(live) && !storage::exists(dead));
  CHECK(storage::stale_pending(live, -1) == false && storage::stale_pending(live, 0) == false);
  // a dead pid of THIS pid namespace is stale; the same dead pid written from another namespace
  // (another container sharing the cache: invisible to kill) only ages out
  const std::string ns = live.substr(live.rfind("-n") + 2, 12);
  const std::string dead_here = live.substr(0, live.rfind(".p")) + ".p999999999-1-n" + ns + ".unverified";
  const std::string foreign = live.substr(0, live.rfind(".p")) + ".p999999999-2-nforeign00000.unverified";
  storage::write_file_atomic(dead_here, good.data(), good.size(), false);
  storage::write_file_atomic(foreign, good.data(), good.size(), false);
  CHECK(storage::stale_pending(dead_here, 3600) && !storage::stale_pending(foreign, 3600));
  struct timespec old_t[2] = {{0, 0}, {::time(nullptr) - 7200, 0}};
  old_t[0] = old_t[1];
  CHECK(::utimensat(AT_FDCWD, foreign.c_str(), old_t, 0) == 0);
  CHECK(storage::stale_pending(foreign, 3600));
  CHECK(cache.sweep_pending(3600) == 2 && storage::exists(live));
}

TEST(lz4_decoder_exact_buffers_and_corrupt_input) {
  // The decoder's fast paths copy 8/16 bytes at a time inside checked slack: round trips into
  // exact-size heap buffers (an ASan build catches any byte past them) and corrupt / truncated
  // blocks that must raise or stay in bounds (python tools/build.py --asan && build/asan/core_tests).
  std::mt19937_64 rng(7);
  for (int it = 0; it < 1500; ++it) {
    const size_t n = rng() % 70000;
    std::vector<uint8_t> d(n);
    const int kind = it % 5;
    for (size_t i = 0; i < n; ++i) {
      if (kind == 0) d[i] = uint8_t(rng());
      else if (kind == 1) d[i] = uint8_t(rng() % 3);
      else if (kind == 2) d[i] = uint8_t((i % (1 + it % 7)) * 17);
      else if (kind == 3) d[i] = 0;
      else d[i] = (rng() % 4 == 0) ? uint8_t(rng()) : (i ? d[i - 1] : 1);
    }
    std::vector<uint8_t> blk(lz4::block_bound(n) + 1);
    const size_t c = n ? lz4::compress_block(d.data(), n, blk.data(), blk.size()) : 0;
    if (n) {
      std::vector<uint8_t> out(n);
      CHECK(lz4::decompress_block(blk.data(), c, out.data(), 0, n) == n && out == d);
    }
    std::vector<uint8_t> bad(blk.begin(), blk.begin() + (c ? c : 1));
    for (int k = 0; k < 3 && !bad.empty(); ++k) bad[rng() % bad.size()] ^= uint8_t(1 + rng() % 255);
    const size_t cut = bad.empty() ? 0 : rng() % (bad.size() + 1);
    const size_t cap = 1 + rng() % (n + 64);
    std::vector<uint8_t> src(bad.begin(), bad.begin() + cut), out(cap);
    try {
      CHECK(lz4::decompress_block(src.data(), src.size(), out.data(), 0, cap) <= cap);
    } catch (const std::exception&) {
    }
  }
}

TEST(copy_ranges_skip_holes) {
  using R = std::vector<std::pair<uint64_t, uint64_t>>;
  // three reserved regions of 100 bytes holding runs of 90, 0 and 70 bytes; one run starts mid-region
  CHECK((zest::copy_ranges({0, 100, 210}, {90, 0, 70}, 0) == R{{0, 90}, {210, 280}}));
  // gaps of at most max_gap merge; out-of-order input is sorted first
  CHECK((zest::copy_ranges({210, 0}, {70, 90}, 120) == R{{0, 280}}));
  CHECK((zest::copy_ranges({0, 95}, {90, 5}, 5) == R{{0, 100}}));
  CHECK((zest::copy_ranges({0, 96}, {90, 5}, 5) == R{{0, 90}, {96, 101}}));
  CHECK(zest::copy_ranges({}, {}, 1).empty());
}

TEST(peer_pool_leases) {
  // Lease accounting of the connection pool against a loopback seeding server: a lease raises its
  // session's user count by exactly one for its lifetime, busy sessions make the pool open more
  // connections up to the per-peer limit, and idle sessions are handed out one per caller.
  char tmpl[] = "/tmp/zest_cpp_pool_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  setenv("ZEST_CACHE_DIR", dir, 1);
  Config cfg = Config::from_env();
  storage::XorbCache cache(cfg);
  bt::BtServer srv(cfg, &cache, {}, 0);
  srv.start();
  const net::Addr a = net::Addr::parse("127.0.0.1:" + std::to_string(srv.port()), 6881);
  Sha1Digest ih{};
  bt::PeerPool pool(cfg.peer_id, 0, 64, 5000, 4);
  std::vector<std::shared_ptr<bt::PeerSession>> held;
  for (int i = 0; i < 4; ++i) held.push_back(pool.get_or_connect(a, ih));
  CHECK(pool.count(a) == 4);
  std::vector<bt::PeerSession*> raw;
  for (auto& h : held) {
    CHECK(h->users() == 1);
    raw.push_back(h.get());
  }
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 4; ++j) CHECK(raw[i] != raw[j]);
  held.clear();
  for (auto* r : raw) CHECK(r->users() == 0);
  // many sequential lease/release cycles keep the count at zero, and concurrent holders still get
  // distinct sessions (before the fix every cycle drove the session one lower)
  for (int k = 0; k < 10; ++k) (void)pool.get_or_connect(a, ih);
  for (auto* r : raw) CHECK(r->users() == 0);
  for (int i = 0; i < 4; ++i) held.push_back(pool.get_or_connect(a, ih));
  CHECK(pool.count(a) == 4);
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 4; ++j) CHECK(held[i].get() != held[j].get());
  held.clear();
  srv.stop();
}

int main() {
  for (auto& [name, fn] : registry()) {
    const int before = g_failed;
    try {
      fn();
    } catch (const std::exception& e) {
      ++g_failed;
      std::fprintf(stderr, "  EXCEPTION in %s: %s\n", name, e.what());
    }
    std::printf("%s %s\n", g_failed == before ? "PASS" : "FAIL", name);
  }
  std::printf("%d checks, %d failed\n", g_checks, g_failed);
  return g_failed ? 1 : 0;
}
