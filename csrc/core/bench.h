// `zest bench --synthetic`: host micro-benchmarks of the protocol hot paths.
//
// Reference: src/bench.zig:150-283 — five rows (bencode_encode, bencode_decode, blake3_64kb,
// sha1_info_hash, bt_wire_frame) with the JSON schema {"results":[{"name","runs","median_ns",
// "throughput_mbps","bytes_processed"}]}.  The reference reports mean-as-"median" (total/runs,
// bench.zig:23-26); here runs are timed in batches and the reported median_ns is the true median of
// per-batch means, throughput_mbps is MiB/s over the whole run.  Extra rows cover the Xet data path
// this framework adds on the host (keyed chunk hash, LZ4 decode, CDC, Merkle).
#pragma once

#include <cstdint>
#include <ostream>
#include <string>
#include <vector>

namespace zest::bench {

struct Result {
  std::string name;
  uint32_t runs = 0;
  double median_ns = 0;  // per-operation median over batches; fractional for sub-ns operations
  uint64_t total_ns = 0;
  uint64_t bytes_processed = 0;
  double throughput_mbps() const;  // MiB/s
};

// `extended` adds the Xet data-path rows after the reference's five.
std::vector<Result> run_synthetic(bool extended = true);
void write_text(std::ostream& os, const std::vector<Result>& r);
void write_json(std::ostream& os, const std::vector<Result>& r);

}  // namespace zest::bench
