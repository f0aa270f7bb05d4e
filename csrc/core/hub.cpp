#include "hub.h"

#include <algorithm>

#include <fcntl.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstring>
#include <map>
#include <mutex>

#include "json.h"
#include "storage.h"

namespace zest::hub {

http::Headers auth_headers(const Config& cfg) {
  http::Headers h;
  if (cfg.hf_token) h.emplace_back("Authorization", "Bearer " + *cfg.hf_token);
  return h;
}

namespace {
std::string api_base(const Config& cfg, const std::string& type) { return cfg.hub_url + "/api/" + type + "s/"; }

void add_files(const json::Value& arr, std::vector<RepoFile>& out) {
  for (const auto& e : arr.array()) {
    if (e.str_or("type", "file") != "file") continue;
    RepoFile f;
    f.path = e.str_or("path", "");
    if (f.path.empty()) f.path = e.str_or("rfilename", "");
    f.size = uint64_t(e.int_or("size", 0));
    std::string xh = e.str_or("xetHash", "");
    if (xh.empty() && e["xet"].is_object()) xh = e["xet"].str_or("hash", "");
    if (!xh.empty()) f.xet_hash = xh;
    if (!f.path.empty()) out.push_back(std::move(f));
  }
}
}  // namespace

std::vector<RepoFile> list_files(const Config& cfg, const std::string& repo_id, const std::string& revision,
                                 const std::string& repo_type) {
  std::vector<RepoFile> out;
  std::string url = api_base(cfg, repo_type) + repo_id + "/tree/" + http::percent_encode(
      reinterpret_cast<const uint8_t*>(revision.data()), revision.size()) + "?recursive=true&expand=true";
  for (int page = 0; page < 1000 && !url.empty(); ++page) {
    http::Response r = http::get(url, auth_headers(cfg));
    if (r.status == 401 || r.status == 403) throw Error("Unauthorized", "listing " + repo_id);
    if (r.status == 404) throw Error("RepoNotFound", repo_id + "@" + revision);
    if (r.status != 200) throw Error("HttpError", "tree status " + std::to_string(r.status));
    add_files(json::Value::parse(r.body), out);
    // RFC 5988 pagination: Link: <url>; rel="next"
    std::string link = r.header("link");
    url.clear();
    size_t nx = link.find("rel=\"next\"");
    if (nx != std::string::npos) {
      size_t lt = link.rfind('<', nx), gt = link.find('>', lt);
      if (lt != std::string::npos && gt != std::string::npos) url = link.substr(lt + 1, gt - lt - 1);
    }
  }
  return out;
}

std::optional<std::string> extract_json_sha(std::string_view j) {
  static const std::string_view needle = "\"sha\":\"";
  size_t p = j.find(needle);
  if (p == std::string_view::npos) return std::nullopt;
  p += needle.size();
  if (p + 40 > j.size()) return std::nullopt;
  for (size_t i = 0; i < 40; ++i)
    if (!std::isxdigit(static_cast<unsigned char>(j[p + i]))) return std::nullopt;
  return std::string(j.substr(p, 40));
}

std::optional<std::string> resolve_commit(const Config& cfg, const std::string& repo_id, const std::string& revision,
                                          const std::string& repo_type) {
  try {
    http::Response r = http::get(api_base(cfg, repo_type) + repo_id + "/revision/" + revision, auth_headers(cfg));
    if (r.status != 200) return std::nullopt;
    if (auto fast = extract_json_sha(r.body)) return fast;
    // Not compact JSON: parse properly.
    std::string sha = json::Value::parse(r.body).str_or("sha", "");
    if (sha.size() == 40 && std::all_of(sha.begin(), sha.end(), [](char c) { return std::isxdigit(uint8_t(c)); }))
      return sha;
    return std::nullopt;
  } catch (const Error&) {
    return std::nullopt;
  }
}

XetToken xet_read_token(const Config& cfg, const std::string& repo_id, const std::string& revision,
                        const std::string& repo_type) {
  http::Response r = http::get(api_base(cfg, repo_type) + repo_id + "/xet-read-token/" + revision, auth_headers(cfg));
  if (r.status == 401 || r.status == 403) throw Error("Unauthorized", "xet-read-token");
  if (r.status != 200) throw Error("HttpError", "xet-read-token status " + std::to_string(r.status));
  json::Value v = json::Value::parse(r.body);
  XetToken t;
  t.access_token = v.str_or("accessToken", "");
  t.cas_url = v.str_or("casUrl", "");
  t.exp = v.int_or("exp", 0);
  if (t.cas_url.empty()) {  // header form used by the Hub for some endpoints
    t.cas_url = r.header("x-xet-cas-url");
    t.access_token = r.header("x-xet-access-token");
  }
  if (t.cas_url.empty() || t.access_token.empty()) throw Error("XetAuthFailed", "no casUrl/accessToken");
  while (!t.cas_url.empty() && t.cas_url.back() == '/') t.cas_url.pop_back();
  return t;
}

uint64_t download_regular(const Config& cfg, const std::string& repo_id, const std::string& revision,
                          const std::string& path, const std::string& out_path) {
  const size_t slash = out_path.rfind('/');
  if (slash != std::string::npos) storage::ensure_dir(out_path.substr(0, slash));
  const std::string tmp = out_path + ".incomplete";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw Error("IoError", tmp + ": " + std::strerror(errno));
  uint64_t total = 0;
  http::RequestOptions opt;
  opt.timeout_ms = 120000;
  opt.sink = [&](const uint8_t* p, size_t n) {
    while (n) {
      ssize_t w = ::write(fd, p, n);
      if (w < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      p += w;
      n -= size_t(w);
      total += uint64_t(w);
    }
    return true;
  };
  http::Response r;
  try {
    r = http::get(cfg.hub_url + "/" + repo_id + "/resolve/" + revision + "/" + path, auth_headers(cfg), opt);
  } catch (...) {
    ::close(fd);
    ::unlink(tmp.c_str());
    throw;
  }
  ::fdatasync(fd);
  ::close(fd);
  if (r.status != 200) {
    ::unlink(tmp.c_str());
    throw Error("HttpError", "resolve " + path + " status " + std::to_string(r.status));
  }
  if (::rename(tmp.c_str(), out_path.c_str()) != 0) throw Error("IoError", "rename " + out_path);
  return total;
}

}  // namespace zest::hub

namespace zest::cas {

uint64_t Reconstruction::total_unpacked() const {
  uint64_t t = 0;
  for (auto& x : terms) t += x.unpacked_length;
  return t;
}

const FetchInfo* Reconstruction::match(const std::string& hex, uint64_t start, uint64_t end) const {
  auto it = fetch_info.find(hex);
  if (it == fetch_info.end()) return nullptr;
  for (const auto& fi : it->second)
    if (fi.range.start <= start && fi.range.end >= end) return &fi;
  return nullptr;
}

Reconstruction parse_reconstruction(std::string_view text) {
  json::Value v = json::Value::parse(text);
  Reconstruction r;
  r.offset_into_first_range = uint64_t(v.int_or("offset_into_first_range", 0));
  for (const auto& t : v["terms"].array()) {
    Term term;
    term.hash_hex = t.str_or("hash", "");
    term.hash = xet::from_hex(term.hash_hex);
    term.unpacked_length = uint64_t(t.int_or("unpacked_length", 0));
    term.range.start = uint64_t(t["range"].int_or("start", 0));
    term.range.end = uint64_t(t["range"].int_or("end", 0));
    if (term.range.end < term.range.start) throw Error("InvalidReconstruction", "bad term range");
    r.terms.push_back(std::move(term));
  }
  for (const auto& kv : v["fetch_info"].object()) {
    auto& vec = r.fetch_info[kv.first];
    for (const auto& e : kv.second.array()) {
      FetchInfo fi;
      fi.range.start = uint64_t(e["range"].int_or("start", 0));
      fi.range.end = uint64_t(e["range"].int_or("end", 0));
      fi.url = e.str_or("url", "");
      fi.url_range.start = uint64_t(e["url_range"].int_or("start", 0));
      fi.url_range.end = uint64_t(e["url_range"].int_or("end", 0));
      vec.push_back(std::move(fi));
    }
  }
  return r;
}

std::string reconstruction_to_json(const Reconstruction& r) {
  json::Writer w;
  w.obj().key("offset_into_first_range").num_u(r.offset_into_first_range).key("terms").arr();
  for (auto& t : r.terms) {
    w.obj().key("hash").str(t.hash_hex).key("unpacked_length").num_u(t.unpacked_length);
    w.key("range").obj().key("start").num_u(t.range.start).key("end").num_u(t.range.end).end().end();
  }
  w.end().key("fetch_info").obj();
  for (auto& kv : r.fetch_info) {
    w.key(kv.first).arr();
    for (auto& fi : kv.second) {
      w.obj().key("range").obj().key("start").num_u(fi.range.start).key("end").num_u(fi.range.end).end();
      w.key("url").str(fi.url);
      w.key("url_range").obj().key("start").num_u(fi.url_range.start).key("end").num_u(fi.url_range.end).end();
      w.end();
    }
    w.end();
  }
  w.end().end();
  return w.out();
}

Reconstruction CasClient::get_reconstruction(const std::string& file_hash_hex) const {
  http::Headers h{{"Authorization", "Bearer " + token_}};
  for (const char* ver : {"/v1/reconstructions/", "/reconstruction/"}) {
    http::Response r = http::get(url_ + ver + file_hash_hex, h);
    if (r.status == 404) continue;
    if (r.status == 401 || r.status == 403) throw Error("Unauthorized", "cas reconstruction");
    if (r.status != 200) throw Error("HttpError", "reconstruction status " + std::to_string(r.status));
    return parse_reconstruction(r.body);
  }
  throw Error("FileNotFound", file_hash_hex);
}

Bytes CasClient::fetch(const FetchInfo& fi, int timeout_ms) const {
  if (fi.url_range.end < fi.url_range.start || fi.url_range.end - fi.url_range.start >= (uint64_t(1) << 40))
    throw Error("InvalidRange", "xorb url_range " + std::to_string(fi.url_range.start) + "-" +
                                    std::to_string(fi.url_range.end));
  const uint64_t want = fi.url_range.end - fi.url_range.start + 1;
  if (is_mem_url(fi.url)) {
    const uint8_t* p = mem_origin_find(fi.url, fi.url_range.start, fi.url_range.end);
    if (!p) throw Error("HttpError", "xorb fetch status 404 (memory origin has no run at " + fi.url + ")");
    return Bytes(p, p + want);
  }
  http::RequestOptions opt;
  opt.timeout_ms = timeout_ms;
  Bytes out;
  out.reserve(size_t(want));
  opt.sink = [&](const uint8_t* p, size_t n) {
    out.insert(out.end(), p, p + n);
    return true;
  };
  // Presigned URLs carry their own auth; the CAS itself (our fake, or direct CAS URLs) takes the token.
  http::Headers h;
  if (fi.url.rfind(url_, 0) == 0) h.emplace_back("Authorization", "Bearer " + token_);
  http::Response r = http::get_range(fi.url, fi.url_range.start, fi.url_range.end, h, opt);
  if (r.status != 200 && r.status != 206) throw Error("HttpError", "xorb fetch status " + std::to_string(r.status));
  if (r.status == 200 && out.size() > want) {
    // Server ignored Range: slice it ourselves (the whole object must reach past the range).
    if (out.size() - want < fi.url_range.start) throw Error("ShortRead", "xorb object shorter than its range");
    Bytes s(out.begin() + long(fi.url_range.start), out.begin() + long(fi.url_range.start + want));
    return s;
  }
  if (out.size() != want) throw Error("ShortRead", "xorb range length mismatch");
  return out;
}

size_t CasClient::fetch_into(const FetchInfo& fi, uint8_t* dst, size_t room, int timeout_ms) const {
  if (fi.url_range.end < fi.url_range.start) throw Error("InvalidRange", "xorb url_range end before start");
  const uint64_t want = fi.url_range.end - fi.url_range.start + 1;
  if (!dst || want > room) return 0;
  if (is_mem_url(fi.url)) {
    const uint8_t* p = mem_origin_find(fi.url, fi.url_range.start, fi.url_range.end);
    if (!p) throw Error("HttpError", "xorb fetch status 404 (memory origin has no run at " + fi.url + ")");
    std::memcpy(dst, p, want);
    return size_t(want);
  }
  http::RequestOptions opt;
  opt.timeout_ms = timeout_ms;
  uint64_t pos = 0;
  bool overflow = false;
  opt.sink = [&](const uint8_t* p, size_t n) {
    if (pos + n > want) {  // a server that ignored Range: stop reading, fall back to fetch()
      overflow = true;
      return false;
    }
    std::memcpy(dst + pos, p, n);
    pos += n;
    return true;
  };
  http::Headers h;
  if (fi.url.rfind(url_, 0) == 0) h.emplace_back("Authorization", "Bearer " + token_);
  http::Response r;
  try {
    r = http::get_range(fi.url, fi.url_range.start, fi.url_range.end, h, opt);
  } catch (const Error& e) {
    if (overflow) return 0;
    throw;
  }
  if (overflow) return 0;
  if (r.status == 200) return fi.url_range.start == 0 && pos == want ? size_t(pos) : 0;  // whole body = range
  if (r.status != 206) throw Error("HttpError", "xorb fetch status " + std::to_string(r.status));
  if (pos != want) throw Error("ShortRead", "xorb range length mismatch");
  return size_t(pos);
}

namespace {
struct MemRun {
  const uint8_t* data;
  uint64_t len;
};
std::mutex g_mem_mu;
std::map<std::pair<std::string, uint64_t>, MemRun> g_mem;  // (xorb hex, url_range.start) -> run
}  // namespace

void mem_origin_add(const std::string& xorb_hex, uint64_t url_start, const uint8_t* data, uint64_t len) {
  std::lock_guard<std::mutex> g(g_mem_mu);
  g_mem[{xorb_hex, url_start}] = MemRun{data, len};
}

void mem_origin_clear() {
  std::lock_guard<std::mutex> g(g_mem_mu);
  g_mem.clear();
}

size_t mem_origin_size() {
  std::lock_guard<std::mutex> g(g_mem_mu);
  return g_mem.size();
}

const uint8_t* mem_origin_find(const std::string& url, uint64_t start, uint64_t end_inclusive) {
  // mem://<name>/<xorb hex>[?query]
  std::string hex = url.substr(url.rfind('/') + 1);
  hex = hex.substr(0, hex.find('?'));
  std::lock_guard<std::mutex> g(g_mem_mu);
  auto it = g_mem.upper_bound({hex, start});
  if (it == g_mem.begin()) return nullptr;
  --it;  // the run starting at or before `start`
  if (it->first.first != hex || end_inclusive < start) return nullptr;
  // [start, end_inclusive] inside [run_start, run_start + len), without overflowing on a hostile range
  const uint64_t skip = start - it->first.second, len = it->second.len;
  if (skip >= len || end_inclusive - start >= len - skip) return nullptr;
  return it->second.data + skip;
}

}  // namespace zest::cas
