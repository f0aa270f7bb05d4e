#include "http.h"

#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>

namespace zest::http {

namespace {

std::string lower(std::string_view s) {
  std::string o(s);
  for (auto& c : o) c = char(std::tolower(static_cast<unsigned char>(c)));
  return o;
}

bool ieq(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i]))) return false;
  return true;
}

SSL_CTX* tls_ctx(bool insecure) {
  static std::once_flag once;
  static SSL_CTX* ctx_verify = nullptr;
  static SSL_CTX* ctx_insecure = nullptr;
  std::call_once(once, [] {
    OPENSSL_init_ssl(0, nullptr);
    ctx_verify = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_default_verify_paths(ctx_verify);
    SSL_CTX_set_verify(ctx_verify, SSL_VERIFY_PEER, nullptr);
    ctx_insecure = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_verify(ctx_insecure, SSL_VERIFY_NONE, nullptr);
  });
  return insecure ? ctx_insecure : ctx_verify;
}

// One client connection: plain TCP or TLS.
class Conn {
 public:
  Conn(const Url& u, int timeout_ms, bool insecure) {
    net::Addr a = net::Addr::resolve(u.host, u.port);
    sock_ = net::Socket::connect_tcp(a, timeout_ms);
    sock_.set_timeout(timeout_ms);
    if (u.scheme == "https") {
      ssl_ = SSL_new(tls_ctx(insecure));
      SSL_set_fd(ssl_, sock_.fd());
      SSL_set_tlsext_host_name(ssl_, u.host.c_str());
      if (!insecure) SSL_set1_host(ssl_, u.host.c_str());
      if (SSL_connect(ssl_) != 1) {
        unsigned long e = ERR_get_error();
        char buf[256];
        ERR_error_string_n(e, buf, sizeof(buf));
        throw Error("TlsError", std::string(u.host) + ": " + buf);
      }
    }
  }
  ~Conn() {
    if (ssl_) {
      SSL_shutdown(ssl_);
      SSL_free(ssl_);
    }
  }
  void write(const void* p, size_t n) {
    if (!ssl_) return sock_.write_all(p, n);
    const uint8_t* b = static_cast<const uint8_t*>(p);
    while (n) {
      int w = SSL_write(ssl_, b, int(std::min<size_t>(n, 1 << 30)));
      if (w <= 0) throw Error("WriteFailed", "tls write");
      b += w;
      n -= size_t(w);
    }
  }
  size_t read(void* p, size_t n) {
    if (!ssl_) return sock_.read_some(p, n);
    int r = SSL_read(ssl_, p, int(std::min<size_t>(n, 1 << 30)));
    if (r > 0) return size_t(r);
    int e = SSL_get_error(ssl_, r);
    if (e == SSL_ERROR_ZERO_RETURN || e == SSL_ERROR_SYSCALL) return 0;
    throw Error("ReadFailed", "tls read");
  }

 private:
  net::Socket sock_;
  SSL* ssl_ = nullptr;
};

// Buffered reader over a Conn.
class Reader {
 public:
  explicit Reader(Conn& c) : c_(c) { buf_.reserve(1 << 16); }
  bool fill() {
    if (pos_ > 0 && pos_ == buf_.size()) {
      buf_.clear();
      pos_ = 0;
    }
    const size_t old = buf_.size();
    buf_.resize(old + (1 << 16));
    size_t n = c_.read(buf_.data() + old, 1 << 16);
    buf_.resize(old + n);
    return n > 0;
  }
  std::string line() {
    while (true) {
      auto it = std::search(buf_.begin() + long(pos_), buf_.end(), kCrlf, kCrlf + 2);
      if (it != buf_.end()) {
        std::string l(buf_.begin() + long(pos_), it);
        pos_ = size_t(it - buf_.begin()) + 2;
        return l;
      }
      if (buf_.size() - pos_ > (1 << 20)) throw Error("HttpError", "header line too long");
      if (!fill()) throw Error("ConnectionClosed", "while reading headers");
    }
  }
  // Read exactly n bytes into sink.
  void exact(uint64_t n, const Sink& sink) {
    while (n) {
      if (pos_ == buf_.size() && !fill()) throw Error("ConnectionClosed", "truncated body");
      size_t take = size_t(std::min<uint64_t>(n, buf_.size() - pos_));
      if (!sink(reinterpret_cast<const uint8_t*>(buf_.data() + pos_), take)) throw Error("Aborted");
      pos_ += take;
      n -= take;
    }
  }
  void until_close(const Sink& sink) {
    while (true) {
      if (pos_ < buf_.size()) {
        size_t take = buf_.size() - pos_;
        if (!sink(reinterpret_cast<const uint8_t*>(buf_.data() + pos_), take)) throw Error("Aborted");
        pos_ += take;
      }
      if (!fill()) return;
    }
  }

 private:
  static constexpr char kCrlf[2] = {'\r', '\n'};
  Conn& c_;
  std::vector<char> buf_;
  size_t pos_ = 0;
};

Response do_request(const std::string& method, const Url& u, const Headers& headers, std::string_view body,
                    const RequestOptions& opt) {
  Conn c(u, opt.timeout_ms, opt.insecure_tls || std::getenv("ZEST_INSECURE_TLS") != nullptr);
  std::string req = method + " " + u.target + " HTTP/1.1\r\n";
  bool has_host = false, has_ua = false;
  for (auto& h : headers) {
    if (ieq(h.first, "host")) has_host = true;
    if (ieq(h.first, "user-agent")) has_ua = true;
    req += h.first + ": " + h.second + "\r\n";
  }
  if (!has_host) {
    const bool default_port = (u.scheme == "https" && u.port == 443) || (u.scheme == "http" && u.port == 80);
    req += "Host: " + u.host + (default_port ? "" : ":" + std::to_string(u.port)) + "\r\n";
  }
  if (!has_ua) req += "User-Agent: zest/0.4.2\r\n";
  req += "Connection: close\r\n";
  if (!body.empty() || method == "POST" || method == "PUT") req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  req += "\r\n";
  c.write(req.data(), req.size());
  if (!body.empty()) c.write(body.data(), body.size());

  Reader rd(c);
  Response r;
  std::string status = rd.line();
  // HTTP/1.1 200 OK
  size_t sp = status.find(' ');
  if (status.compare(0, 5, "HTTP/") != 0 || sp == std::string::npos) throw Error("HttpError", "bad status line");
  r.status = std::atoi(status.c_str() + sp + 1);
  while (true) {
    std::string l = rd.line();
    if (l.empty()) break;
    size_t colon = l.find(':');
    if (colon == std::string::npos) continue;
    std::string v = l.substr(colon + 1);
    size_t b = v.find_first_not_of(" \t");
    v = b == std::string::npos ? "" : v.substr(b);
    while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.pop_back();
    r.headers.emplace_back(l.substr(0, colon), v);
  }
  const bool redirect = r.status >= 300 && r.status < 400 && !r.header("location").empty();
  Sink sink;
  size_t total = 0;
  if (opt.sink && r.status >= 200 && r.status < 300) {
    sink = opt.sink;
  } else {
    sink = [&](const uint8_t* p, size_t n) {
      total += n;
      if (total > opt.max_body) throw Error("HttpError", "body too large");
      r.body.append(reinterpret_cast<const char*>(p), n);
      return true;
    };
  }
  if (method == "HEAD" || r.status == 204 || r.status == 304) return r;
  const std::string te = lower(r.header("transfer-encoding"));
  const std::string cl = r.header("content-length");
  if (te.find("chunked") != std::string::npos) {
    while (true) {
      std::string szl = rd.line();
      uint64_t sz = std::strtoull(szl.c_str(), nullptr, 16);
      if (sz == 0) {
        while (!rd.line().empty()) {
        }
        break;
      }
      rd.exact(sz, sink);
      rd.line();
    }
  } else if (!cl.empty()) {
    rd.exact(std::strtoull(cl.c_str(), nullptr, 10), redirect ? Sink([](const uint8_t*, size_t) { return true; }) : sink);
  } else {
    rd.until_close(sink);
  }
  return r;
}

}  // namespace

Url Url::parse(std::string_view url) {
  Url u;
  size_t p = url.find("://");
  if (p == std::string_view::npos) throw Error("InvalidUrl", std::string(url));
  u.scheme = lower(url.substr(0, p));
  if (u.scheme != "http" && u.scheme != "https") throw Error("InvalidUrl", "unsupported scheme");
  std::string_view rest = url.substr(p + 3);
  size_t slash = rest.find('/');
  std::string_view hostport = slash == std::string_view::npos ? rest : rest.substr(0, slash);
  u.target = slash == std::string_view::npos ? "/" : std::string(rest.substr(slash));
  size_t at = hostport.rfind('@');
  if (at != std::string_view::npos) hostport = hostport.substr(at + 1);
  u.port = u.scheme == "https" ? 443 : 80;
  if (!hostport.empty() && hostport[0] == '[') {
    size_t e = hostport.find(']');
    u.host = std::string(hostport.substr(1, e - 1));
    if (e + 1 < hostport.size() && hostport[e + 1] == ':') u.port = uint16_t(std::atoi(std::string(hostport.substr(e + 2)).c_str()));
  } else {
    size_t c = hostport.rfind(':');
    if (c != std::string_view::npos) {
      u.host = std::string(hostport.substr(0, c));
      u.port = uint16_t(std::atoi(std::string(hostport.substr(c + 1)).c_str()));
    } else {
      u.host = std::string(hostport);
    }
  }
  if (u.host.empty()) throw Error("InvalidUrl", std::string(url));
  return u;
}

std::string Url::origin() const {
  const bool dflt = (scheme == "https" && port == 443) || (scheme == "http" && port == 80);
  return scheme + "://" + host + (dflt ? "" : ":" + std::to_string(port));
}

std::string percent_encode(const uint8_t* p, size_t n) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  out.reserve(n * 3);
  for (size_t i = 0; i < n; ++i) {
    const uint8_t c = p[i];
    if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
        c == '.' || c == '~') {
      out.push_back(char(c));
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    }
  }
  return out;
}

std::string percent_decode(std::string_view s) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && std::isxdigit(static_cast<unsigned char>(s[i + 1])) &&
        std::isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out.push_back(char(std::stoi(std::string(s.substr(i + 1, 2)), nullptr, 16)));
      i += 2;
      continue;
    }
    out.push_back(s[i] == '+' ? ' ' : s[i]);
  }
  return out;
}

std::string Response::header(std::string_view name) const {
  for (auto& h : headers)
    if (ieq(h.first, name)) return h.second;
  return "";
}

std::string Request::header(std::string_view name) const {
  for (auto& h : headers)
    if (ieq(h.first, name)) return h.second;
  return "";
}

Response request(const std::string& method, const std::string& url, const Headers& headers, std::string_view body,
                 const RequestOptions& opt) {
  std::string cur = url;
  Headers hdrs = headers;
  for (int hop = 0; hop <= opt.max_redirects; ++hop) {
    Url u = Url::parse(cur);
    Response r = do_request(method, u, hdrs, body, opt);
    if (r.status >= 300 && r.status < 400 && !r.header("location").empty() && hop < opt.max_redirects) {
      std::string loc = r.header("location");
      if (loc.rfind("http", 0) != 0) loc = u.origin() + (loc[0] == '/' ? loc : "/" + loc);
      // Do not forward credentials to a different host.
      Url nu = Url::parse(loc);
      if (nu.host != u.host) {
        hdrs.erase(std::remove_if(hdrs.begin(), hdrs.end(), [](auto& h) { return ieq(h.first, "authorization"); }),
                   hdrs.end());
      }
      cur = loc;
      continue;
    }
    return r;
  }
  throw Error("HttpError", "too many redirects");
}

Response get_range(const std::string& url, uint64_t start, uint64_t end_inclusive, const Headers& headers,
                   const RequestOptions& opt) {
  Headers h = headers;
  h.emplace_back("Range", "bytes=" + std::to_string(start) + "-" + std::to_string(end_inclusive));
  return request("GET", url, h, {}, opt);
}

// ---------------------------------------------------------------------------------------------
const char* status_text(int s) {
  switch (s) {
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 206: return "Partial Content";
    case 302: return "Found";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 416: return "Range Not Satisfiable";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Unknown";
  }
}

Server::Server(const net::Addr& bind, Handler handler, int threads) : handler_(std::move(handler)), threads_(threads) {
  listener_ = net::Socket::listen_tcp(bind);
  port_ = listener_.local_addr().port();
}

Server::~Server() { stop(); }

void Server::start() {
  for (int i = 0; i < threads_; ++i) workers_.emplace_back([this] { loop(); });
}

void Server::run() {
  start();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
}

void Server::stop() {
  stop_.store(true);
  listener_.shutdown();
  for (auto& t : workers_)
    if (t.joinable() && t.get_id() != std::this_thread::get_id()) t.join();
  listener_.close();
}

void Server::loop() {
  while (!stop_.load()) {
    net::Addr peer;
    net::Socket s;
    try {
      s = listener_.accept(200, &peer);
    } catch (const Error&) {
      if (stop_.load()) return;
      continue;
    }
    if (!s.valid()) continue;
    try {
      serve(std::move(s), peer);
    } catch (...) {
    }
  }
}

void Server::serve(net::Socket s, net::Addr peer) {
  s.set_timeout(10000);
  std::string buf;
  buf.reserve(8192);
  size_t hdr_end = std::string::npos;
  char tmp[8192];
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    size_t n = s.read_some(tmp, sizeof(tmp));
    if (n == 0) return;
    buf.append(tmp, n);
    if (buf.size() > (1 << 20)) return;
  }
  Request req;
  req.peer = peer;
  size_t le = buf.find("\r\n");
  std::string first = buf.substr(0, le);
  size_t a = first.find(' '), b = first.rfind(' ');
  if (a == std::string::npos || b == a) return;
  req.method = first.substr(0, a);
  req.target = first.substr(a + 1, b - a - 1);
  size_t pos = le + 2;
  while (pos < hdr_end) {
    size_t e = buf.find("\r\n", pos);
    std::string l = buf.substr(pos, e - pos);
    pos = e + 2;
    size_t c = l.find(':');
    if (c == std::string::npos) continue;
    std::string v = l.substr(c + 1);
    size_t st = v.find_first_not_of(" \t");
    req.headers.emplace_back(l.substr(0, c), st == std::string::npos ? "" : v.substr(st));
  }
  size_t q = req.target.find('?');
  req.path = percent_decode(req.target.substr(0, q));
  if (q != std::string::npos) {
    std::string qs = req.target.substr(q + 1);
    size_t p = 0;
    while (p <= qs.size()) {
      size_t amp = qs.find('&', p);
      std::string kv = qs.substr(p, amp == std::string::npos ? std::string::npos : amp - p);
      size_t eq = kv.find('=');
      if (!kv.empty()) req.query[percent_decode(kv.substr(0, eq))] = eq == std::string::npos ? "" : percent_decode(kv.substr(eq + 1));
      if (amp == std::string::npos) break;
      p = amp + 1;
    }
  }
  const std::string cl = req.header("content-length");
  req.body = buf.substr(hdr_end + 4);
  if (!cl.empty()) {
    const size_t want = size_t(std::strtoull(cl.c_str(), nullptr, 10));
    if (want > (size_t(64) << 20)) return;
    while (req.body.size() < want) {
      size_t n = s.read_some(tmp, std::min(sizeof(tmp), want - req.body.size()));
      if (n == 0) return;
      req.body.append(tmp, n);
    }
  }
  requests_.fetch_add(1);
  ServerResponse r;
  try {
    r = handler_(req);
  } catch (const std::exception& e) {
    r.status = 500;
    r.body = std::string("{\"error\":") + "\"internal\"}";
  }
  const uint64_t len = r.stream ? r.stream_len : r.body.size();
  std::string head = "HTTP/1.1 " + std::to_string(r.status) + " " + status_text(r.status) + "\r\n";
  head += "Content-Type: " + r.content_type + "\r\n";
  if (!(r.stream && r.stream_len == ServerResponse::kUntilClose)) head += "Content-Length: " + std::to_string(len) + "\r\n";
  for (auto& h : r.extra) head += h.first + ": " + h.second + "\r\n";
  head += "Connection: close\r\n\r\n";
  s.write_all(head.data(), head.size());
  if (req.method == "HEAD") return;
  if (r.stream) r.stream(s);
  else if (!r.body.empty()) s.write_all(r.body.data(), r.body.size());
}

}  // namespace zest::http
