// HuggingFace Hub API + Xet CAS client.
//
// Reference call sites (zig-xet, not vendored): model_download.listFiles (main.zig:142-154),
// resolveCommitSha (main.zig:638-694), xet-read-token auth (xet_bridge.zig:76-130),
// CasClient.getReconstruction (xet_bridge.zig:133-142) and fetchXorbFromUrl (xet_bridge.zig:196-199),
// downloadRegularFile via /resolve/ (main.zig:696-728; here WITH the auth header and streamed to
// disk instead of buffered in RAM).  Reconstruction paths match xet-core: /v2/reconstructions
// first, then /v1/reconstructions (observed from hf_xet against a logging server).
#pragma once

#include <map>
#include <optional>
#include <string>
#include <vector>

#include "config.h"
#include "http.h"
#include "xet_hash.h"

namespace zest::hub {

struct RepoFile {
  std::string path;
  uint64_t size = 0;
  std::optional<std::string> xet_hash;  // Xet file hash (xet hex); nullopt = regular file
};

http::Headers auth_headers(const Config& cfg);
std::vector<RepoFile> list_files(const Config& cfg, const std::string& repo_id, const std::string& revision,
                                 const std::string& repo_type = "model");
std::optional<std::string> resolve_commit(const Config& cfg, const std::string& repo_id, const std::string& revision,
                                          const std::string& repo_type = "model");
// `"sha":"<40 hex>"` scan (main.zig:781-805 semantics).
std::optional<std::string> extract_json_sha(std::string_view json);

struct XetToken {
  std::string access_token;
  std::string cas_url;
  int64_t exp = 0;
};
XetToken xet_read_token(const Config& cfg, const std::string& repo_id, const std::string& revision,
                        const std::string& repo_type = "model");
// Stream {hub}/{repo}/resolve/{rev}/{path} into out_path (atomic); returns bytes written.
uint64_t download_regular(const Config& cfg, const std::string& repo_id, const std::string& revision,
                          const std::string& path, const std::string& out_path);

}  // namespace zest::hub

namespace zest::cas {

struct Range {
  uint64_t start = 0, end = 0;  // chunk ranges: [start, end); url_range: inclusive end
};

struct FetchInfo {
  Range range;      // chunk index range inside the xorb
  std::string url;
  Range url_range;  // byte range (inclusive end) for the HTTP Range header
};

struct Term {
  xet::Hash hash{};
  std::string hash_hex;
  uint64_t unpacked_length = 0;
  Range range;
};

struct Reconstruction {
  uint64_t offset_into_first_range = 0;
  std::vector<Term> terms;
  std::map<std::string, std::vector<FetchInfo>> fetch_info;  // xet hex -> entries
  uint64_t total_unpacked() const;
  // The fetch_info entry covering [start, end) of xorb `hex` (xet_bridge.zig:221-228).
  const FetchInfo* match(const std::string& hex, uint64_t start, uint64_t end) const;
};

Reconstruction parse_reconstruction(std::string_view json);
std::string reconstruction_to_json(const Reconstruction& r);

class CasClient {
 public:
  CasClient(std::string cas_url, std::string token) : url_(std::move(cas_url)), token_(std::move(token)) {}
  Reconstruction get_reconstruction(const std::string& file_hash_hex) const;
  Bytes fetch(const FetchInfo& fi, int timeout_ms = 120000) const;
  // The url_range straight into caller memory of `room` bytes (a pinned staging region): no
  // intermediate heap buffer.  Returns the bytes written, or 0 when the range does not fit `room`
  // or the server ignored the Range header (the caller falls back to fetch()).
  size_t fetch_into(const FetchInfo& fi, uint8_t* dst, size_t room, int timeout_ms = 120000) const;
  const std::string& url() const { return url_; }

 private:
  std::string url_, token_;
};

// In-process memory origin: fetch_info URLs `mem://<name>/<xorb hex>` are served from host memory
// registered here instead of over HTTP (the bench's CDN stand-in for the public swarm_pull path: the
// same fetch_term waterfall, the bytes copied from pinned host memory like a NIC's DMA into the
// staging buffer, no sockets).  A run is keyed by (xorb hex, url_range.start); a fetch must ask for
// exactly a registered run or a prefix of one.  Registration is process-global and thread-safe.
void mem_origin_add(const std::string& xorb_hex, uint64_t url_start, const uint8_t* data, uint64_t len);
void mem_origin_clear();
size_t mem_origin_size();
// (data, len) of the registered run covering [start, end_inclusive] of `url`'s xorb, or nullptr.
const uint8_t* mem_origin_find(const std::string& url, uint64_t start, uint64_t end_inclusive);
inline bool is_mem_url(const std::string& url) { return url.rfind("mem://", 0) == 0; }

}  // namespace zest::cas
