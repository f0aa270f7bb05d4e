#include "config.h"

#include <algorithm>

#include <cstdlib>
#include <fstream>
#include <sstream>

#include "json.h"

namespace zest {

namespace {
const char* env(const char* k) {
  const char* v = std::getenv(k);
  return (v && *v) ? v : nullptr;
}
std::string trim(std::string s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  size_t b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}
}  // namespace

std::string repo_folder_name(const std::string& repo_id, const std::string& type) {
  std::string s = type + "s--";
  for (char c : repo_id) {
    if (c == '/') s += "--";
    else s.push_back(c);
  }
  return s;
}

Config Config::from_env() {
  Config c;
  c.home = env("HOME") ? env("HOME") : "/root";
  c.hub_url = env("HF_ENDPOINT") ? env("HF_ENDPOINT") : kDefaultHub;
  while (!c.hub_url.empty() && c.hub_url.back() == '/') c.hub_url.pop_back();
  const std::string hf_home = env("HF_HOME") ? env("HF_HOME") : c.home + "/.cache/huggingface";
  c.hf_cache_dir = env("HF_HUB_CACHE") ? env("HF_HUB_CACHE") : hf_home + "/hub";
  c.cache_dir = env("ZEST_CACHE_DIR") ? env("ZEST_CACHE_DIR") : c.home + "/.cache/zest";
  c.xorb_cache_dir = c.cache_dir + "/xorbs";
  c.chunk_cache_dir = c.cache_dir + "/chunks";
  c.pid_file = c.cache_dir + "/zest.pid";
  if (env("HF_TOKEN")) {
    c.hf_token = std::string(env("HF_TOKEN"));
  } else {
    for (const std::string& p : {hf_home + "/token", c.home + "/.cache/huggingface/token"}) {
      std::ifstream f(p);
      if (f) {
        std::stringstream ss;
        ss << f.rdbuf();
        std::string t = trim(ss.str());
        if (!t.empty()) {
          c.hf_token = t;
          break;
        }
      }
    }
  }
  auto port_env = [](const char* k, uint16_t d) -> uint16_t {
    const char* v = env(k);
    if (!v) return d;
    char* end = nullptr;
    long x = std::strtol(v, &end, 10);
    return (end && *end == 0 && x > 0 && x < 65536) ? uint16_t(x) : d;
  };
  c.http_port = port_env("ZEST_HTTP_PORT", kDefaultHttpPort);
  c.listen_port = port_env("ZEST_LISTEN_PORT", kDefaultListenPort);
  c.dht_port = port_env("ZEST_DHT_PORT", kDefaultDhtPort);
  if (const char* b = std::getenv("ZEST_DHT_BOOTSTRAP")) {
    const std::string v = b;
    if (v != "none") {
      size_t p = 0;
      while (p < v.size()) {
        size_t e = v.find(',', p);
        if (e == std::string::npos) e = v.size();
        if (e > p) c.dht_routers.push_back(v.substr(p, e - p));
        p = e + 1;
      }
    }
  } else {
    for (const char* r : kDefaultDhtRouters) c.dht_routers.push_back(r);
  }
  if (const char* v = env("ZEST_MAX_PEERS")) c.max_peers = uint32_t(std::strtoul(v, nullptr, 10));
  if (const char* v = env("ZEST_CACHE_MAX_GB")) c.cache_max_gb = std::max(0.0, std::strtod(v, nullptr));
  if (const char* v = env("ZEST_MAX_INBOUND")) c.max_inbound = uint32_t(std::strtoul(v, nullptr, 10));
  if (const char* v = env("ZEST_PEER_CONNECTIONS")) c.peer_connections = uint32_t(std::strtoul(v, nullptr, 10));
  if (const char* v = env("ZEST_CONCURRENCY")) c.concurrency = std::max(1ul, std::strtoul(v, nullptr, 10));
  if (const char* v = env("ZEST_GPUS")) c.gpus = std::atoi(v);
  if (const char* v = env("ZEST_HBM_CACHE_GB")) c.hbm_cache_gb = std::atof(v);
  if (env("ZEST_TRACE")) c.trace = true;
  if (const char* v = env("ZEST_FAULT")) c.fault = v;
  if (const char* v = env("ZEST_CACHE_WRITES")) c.cache_writes = std::string(v) != "0";
  if (const char* v = env("ZEST_CONNECT_TIMEOUT_MS")) c.connect_timeout_ms = std::atoi(v);
  c.peer_id = peer_id::generate();
  return c;
}

std::string Config::repo_dir(const std::string& repo_id) const { return hf_cache_dir + "/" + repo_folder_name(repo_id); }

std::string Config::snapshot_dir(const std::string& repo_id, const std::string& commit) const {
  return repo_dir(repo_id) + "/snapshots/" + commit;
}

std::string Config::xorb_cache_path(const std::string& key) const {
  if (key.size() < 4) throw Error("InvalidHash", "cache key too short");
  return xorb_cache_dir + "/" + key.substr(0, 2) + "/" + key;
}

std::string Config::chunk_cache_path(const std::string& key) const {
  if (key.size() < 4) throw Error("InvalidHash", "cache key too short");
  return chunk_cache_dir + "/" + key.substr(0, 2) + "/" + key;
}

std::string Config::to_json() const {
  json::Writer w;
  w.obj();
  w.key("version").str(kVersion).key("hub_url").str(hub_url).key("hf_cache_dir").str(hf_cache_dir);
  w.key("cache_dir").str(cache_dir).key("xorb_cache_dir").str(xorb_cache_dir).key("chunk_cache_dir").str(chunk_cache_dir);
  w.key("dht_routers").arr();
  for (const auto& r : dht_routers) w.str(r);
  w.end();
  w.key("pid_file").str(pid_file).key("dht_port").num(int64_t(dht_port)).key("listen_port").num(int64_t(listen_port));
  w.key("http_port").num(int64_t(http_port)).key("max_peers").num(int64_t(max_peers)).key("max_inbound").num(int64_t(max_inbound));
  w.key("peer_connections").num(int64_t(peer_connections)).key("cache_writes").boolean(cache_writes);
  w.key("concurrency").num(int64_t(concurrency)).key("has_token").boolean(hf_token.has_value());
  w.key("gpus").num(int64_t(gpus)).key("hbm_cache_gb").num(hbm_cache_gb, 1);
  w.end();
  return w.out();
}

}  // namespace zest
