#include "bench.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "bencode.h"
#include "blake3.h"
#include "bt_wire.h"
#include "cdc.h"
#include "lz4.h"
#include "sha1.h"
#include "xet_hash.h"

namespace zest::bench {

namespace {

template <class T>
inline void keep(const T& v) {
  asm volatile("" : : "r"(&v) : "memory");
}

uint64_t now_ns() {
  return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now().time_since_epoch())
                      .count());
}

// Run `body` `runs` times in `batches` batches; body returns bytes processed by one run.  A template
// (not std::function) so the per-run cost is the operation itself, as in the reference's loops.
template <class F>
Result measure(const char* name, uint32_t runs, F&& body) {
  const uint32_t batches = std::min<uint32_t>(runs, 25);
  const uint32_t per = runs / batches;
  Result r;
  r.name = name;
  r.runs = per * batches;
  for (uint32_t i = 0; i < std::min<uint32_t>(per, 64); ++i) keep(body());  // warm caches/tables
  // Per-batch time per operation, in fractional ns: a frame write takes well under 1 ns, so an
  // integer division reported it as 0 (round 2).
  std::vector<double> per_run;
  for (uint32_t b = 0; b < batches; ++b) {
    const uint64_t t0 = now_ns();
    for (uint32_t i = 0; i < per; ++i) r.bytes_processed += body();
    const uint64_t dt = now_ns() - t0;
    r.total_ns += dt;
    per_run.push_back(double(dt) / double(per));
  }
  std::nth_element(per_run.begin(), per_run.begin() + per_run.size() / 2, per_run.end());
  r.median_ns = per_run[per_run.size() / 2];
  return r;
}

}  // namespace

double Result::throughput_mbps() const {
  if (!total_ns) return 0;
  return (double(bytes_processed) / (1024.0 * 1024.0)) / (double(total_ns) / 1e9);
}

std::vector<Result> run_synthetic(bool extended) {
  std::vector<Result> out;
  // 1. bencode_encode: the BEP 10 extension handshake dict.
  {
    std::string buf;
    buf.reserve(64);
    out.push_back(measure("bencode_encode", 10000, [&]() -> uint64_t {
      buf.clear();
      bencode::Encoder e(buf);
      e.begin_dict().key("m").begin_dict().key("ut_xet").integer(1).end();
      e.key("p").integer(6881).key("v").str("zest/0.4").end();
      keep(buf);
      return buf.size();
    }));
  }
  // 2. bencode_decode of the same document.
  {
    static const std::string_view in = "d1:md6:ut_xeti1ee1:pi6881e1:v8:zest/0.4e";
    bencode::Document doc;
    out.push_back(measure("bencode_decode", 10000, [&]() -> uint64_t {
      doc.parse(in);
      keep(doc);
      return in.size();
    }));
  }
  // 3. blake3_64kb: plain BLAKE3 of a 64 KiB buffer (SIMD tree hashing).
  {
    std::vector<uint8_t> data(65536, 0x42);
    uint8_t h[32];
    out.push_back(measure("blake3_64kb", 1000, [&]() -> uint64_t {
      blake3::hash(data.data(), data.size(), h);
      keep(h);
      return data.size();
    }));
  }
  // 4. sha1_info_hash: SHA1("zest-xet-v1:" || xorb_hash).
  {
    uint8_t xh[32];
    std::memset(xh, 0xAB, 32);
    out.push_back(measure("sha1_info_hash", 10000, [&]() -> uint64_t {
      auto d = peer_id::info_hash(xh);
      keep(d);
      return 44;
    }));
  }
  // 5. bt_wire_frame: length-prefixed `interested` message with a 64-byte payload.
  {
    uint8_t payload[64];
    std::memset(payload, 0x42, 64);
    alignas(64) uint8_t buf[256];
    out.push_back(measure("bt_wire_frame", 10000, [&]() -> uint64_t {
      const size_t n = bt::write_message(buf, 2 /* interested */, payload, sizeof(payload));
      keep(buf);
      return n;
    }));
  }
  if (!extended) return out;
  // Xet data path rows.
  std::vector<uint8_t> chunk(65536);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& b : chunk) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    b = uint8_t(s >> 56) & 0x3F;  // compressible-ish (6-bit alphabet)
  }
  {
    out.push_back(measure("xet_chunk_hash_64kb", 1000, [&]() -> uint64_t {
      auto h = xet::chunk_hash(chunk.data(), chunk.size());
      keep(h);
      return chunk.size();
    }));
  }
  {
    Bytes frame = lz4::compress_frame(chunk.data(), chunk.size());
    std::vector<uint8_t> dst(chunk.size());
    out.push_back(measure("lz4_decode_64kb", 1000, [&]() -> uint64_t {
      lz4::decompress_frame_into(frame.data(), frame.size(), dst.data(), dst.size());
      keep(dst);
      return dst.size();
    }));
  }
  {
    // bf16 weights as Xet stores them: N(0, 0.02) values (sum of 4 uniforms, scaled), BG4-LZ4 --
    // the host pull's decode path for real checkpoints (exponent planes: ~7000 short sequences per
    // 64 KiB chunk)
    std::vector<uint8_t> w(65536);
    for (size_t i = 0; i + 1 < w.size(); i += 2) {
      float u = 0;
      for (int k = 0; k < 4; ++k) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        u += float(s >> 40) / float(1ull << 24) - 0.5f;
      }
      const float v = u * 0.02f * 1.7320508f;
      uint32_t bits;
      std::memcpy(&bits, &v, 4);
      w[i] = uint8_t(bits >> 16);
      w[i + 1] = uint8_t(bits >> 24);
    }
    Bytes payload;
    const xet::Scheme sc = xet::compress_chunk(w.data(), w.size(), xet::CompressionPolicy::BG4, payload);
    std::vector<uint8_t> dst(w.size());
    out.push_back(measure("bg4_lz4_decode_bf16_64kb", 1000, [&]() -> uint64_t {
      xet::decompress_chunk(sc, payload.data(), payload.size(), dst.data(), dst.size());
      keep(dst);
      return dst.size();
    }));
  }
  {
    std::vector<uint8_t> big(8u << 20);
    for (auto& b : big) {
      s ^= s << 13, s ^= s >> 7, s ^= s << 17;
      b = uint8_t(s >> 56);
    }
    out.push_back(measure("cdc_chunk_8mb", 50, [&]() -> uint64_t {
      auto e = xet::chunk_ends(big.data(), big.size());
      keep(e);
      return big.size();
    }));
    std::vector<xet::HashSize> leaves;
    auto ends = xet::chunk_ends(big.data(), big.size());
    uint64_t prev = 0;
    for (uint64_t e : ends) {
      leaves.push_back({xet::chunk_hash(big.data() + prev, e - prev), e - prev});
      prev = e;
    }
    out.push_back(measure("merkle_file_hash_8mb", 200, [&]() -> uint64_t {
      auto h = xet::file_hash(leaves);
      keep(h);
      return big.size();
    }));
  }
  return out;
}

void write_text(std::ostream& os, const std::vector<Result>& r) {
  char line[160];
  os << "\nzest benchmark results (blake3: " << blake3::simd_backend() << ")\n";
  std::snprintf(line, sizeof line, "%22s %10s %12s %12s\n", "Name", "Runs", "Median (ns)", "MB/s");
  os << line;
  std::snprintf(line, sizeof line, "%22s %10s %12s %12s\n", "----------------------", "----------",
                "------------", "------------");
  os << line;
  for (auto& x : r) {
    std::snprintf(line, sizeof line, "%22s %10u %12.2f %12.1f\n", x.name.c_str(), x.runs,
                  x.median_ns, x.throughput_mbps());
    os << line;
  }
  os << "\n";
}

void write_json(std::ostream& os, const std::vector<Result>& r) {
  os << "{\"results\":[";
  char buf[256];
  for (size_t i = 0; i < r.size(); ++i) {
    std::snprintf(buf, sizeof buf,
                  "%s{\"name\":\"%s\",\"runs\":%u,\"median_ns\":%.3f,\"throughput_mbps\":%.1f,\"bytes_processed\":%llu}",
                  i ? "," : "", r[i].name.c_str(), r[i].runs, r[i].median_ns,
                  r[i].throughput_mbps(), (unsigned long long)r[i].bytes_processed);
    os << buf;
  }
  os << "]}\n";
}

}  // namespace zest::bench
