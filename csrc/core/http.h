// HTTP/1.1 client (plain + TLS via OpenSSL, redirects, chunked bodies, Range requests, streaming
// sinks) and a small threaded HTTP/1.1 server with a router.
//
// Replaces the reference's std.http usage: HF Hub API + /resolve/ downloads (main.zig:638-728),
// the BT tracker GET (bt_tracker.zig:65-107), the Xet CAS/CDN ranged GETs (zig-xet), the local
// REST API server (http_api.zig:48-114) and the Python client's health checks.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <utility>
#include <vector>

#include "common.h"
#include "net.h"

namespace zest::http {

struct Url {
  std::string scheme;  // http | https
  std::string host;
  uint16_t port = 0;
  std::string target;  // path + query
  static Url parse(std::string_view url);  // throws Error("InvalidUrl")
  std::string origin() const;              // scheme://host[:port]
};

std::string percent_encode(const uint8_t* p, size_t n);  // RFC 3986 unreserved kept, uppercase hex
std::string percent_decode(std::string_view s);

using Headers = std::vector<std::pair<std::string, std::string>>;

struct Response {
  int status = 0;
  Headers headers;
  std::string body;
  std::string header(std::string_view name) const;  // case-insensitive, "" if absent
};

// Body sink for streaming large responses: called with each piece; return false to abort.
using Sink = std::function<bool(const uint8_t*, size_t)>;

struct RequestOptions {
  int timeout_ms = 30000;
  int max_redirects = 5;
  size_t max_body = size_t(1) << 34;  // 16 GiB safety cap for buffered bodies
  Sink sink;                          // if set, body is streamed here instead of buffered
  bool insecure_tls = false;          // skip certificate verification (tests/proxies)
};

Response request(const std::string& method, const std::string& url, const Headers& headers = {},
                 std::string_view body = {}, const RequestOptions& opt = {});
inline Response get(const std::string& url, const Headers& headers = {}, const RequestOptions& opt = {}) {
  return request("GET", url, headers, {}, opt);
}
// Inclusive byte range, as Xet fetch_info url_range.
Response get_range(const std::string& url, uint64_t start, uint64_t end_inclusive, const Headers& headers = {},
                   const RequestOptions& opt = {});

// ---------------------------------------------------------------------------------------------
struct Request {
  std::string method;
  std::string target;  // raw
  std::string path;    // decoded path without query
  std::map<std::string, std::string> query;
  Headers headers;
  std::string body;
  net::Addr peer;
  std::string header(std::string_view name) const;
};

struct ServerResponse {
  int status = 200;
  std::string content_type = "application/json";
  std::string body;
  Headers extra;
  // Optional streamed body (e.g. a file range): producer writes to the socket via the callback.
  // stream_len == kUntilClose: no Content-Length, the body ends when the connection closes (SSE).
  std::function<void(net::Socket&)> stream;
  uint64_t stream_len = 0;
  static constexpr uint64_t kUntilClose = ~uint64_t(0);
};

using Handler = std::function<ServerResponse(const Request&)>;

class Server {
 public:
  Server(const net::Addr& bind, Handler handler, int threads = 8);
  ~Server();
  void start();  // background accept threads
  void run();    // block until stop()
  void stop();
  uint16_t port() const { return port_; }
  bool running() const { return !stop_.load(); }
  uint64_t requests() const { return requests_.load(); }

 private:
  void loop();
  void serve(net::Socket s, net::Addr peer);
  net::Socket listener_;
  Handler handler_;
  int threads_;
  uint16_t port_ = 0;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> requests_{0};
  std::vector<std::thread> workers_;
};

const char* status_text(int status);

}  // namespace zest::http
