#include "net.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>
#include <cstring>

namespace zest::net {

namespace {
[[noreturn]] void sys_fail(const char* what) { throw Error("NetworkError", std::string(what) + ": " + std::strerror(errno)); }

bool poll_fd(int fd, short ev, int timeout_ms) {
  pollfd p{fd, ev, 0};
  while (true) {
    int r = ::poll(&p, 1, timeout_ms);
    if (r > 0) return true;
    if (r == 0) return false;
    if (errno != EINTR) sys_fail("poll");
  }
}
}  // namespace

Addr Addr::parse(std::string_view hp, uint16_t default_port) {
  std::string host;
  uint16_t port = default_port;
  if (!hp.empty() && hp[0] == '[') {
    size_t e = hp.find(']');
    if (e == std::string_view::npos) throw Error("InvalidAddress", std::string(hp));
    host = std::string(hp.substr(1, e - 1));
    if (e + 1 < hp.size() && hp[e + 1] == ':') port = uint16_t(std::stoi(std::string(hp.substr(e + 2))));
  } else {
    size_t c = hp.rfind(':');
    if (c != std::string_view::npos && hp.find(':') == c) {
      host = std::string(hp.substr(0, c));
      int p = 0;
      try {
        p = std::stoi(std::string(hp.substr(c + 1)));
      } catch (...) {
        throw Error("InvalidAddress", std::string(hp));
      }
      if (p < 0 || p > 65535) throw Error("InvalidAddress", std::string(hp));
      port = uint16_t(p);
    } else {
      host = std::string(hp);
    }
  }
  if (host.empty()) throw Error("InvalidAddress", std::string(hp));
  return resolve(host, port);
}

Addr Addr::resolve(std::string_view host, uint16_t port) {
  Addr a;
  std::string h(host);
  sockaddr_in v4{};
  if (inet_pton(AF_INET, h.c_str(), &v4.sin_addr) == 1) {
    v4.sin_family = AF_INET;
    v4.sin_port = htons(port);
    std::memcpy(&a.ss, &v4, sizeof(v4));
    a.len = sizeof(v4);
    return a;
  }
  sockaddr_in6 v6{};
  if (inet_pton(AF_INET6, h.c_str(), &v6.sin6_addr) == 1) {
    v6.sin6_family = AF_INET6;
    v6.sin6_port = htons(port);
    std::memcpy(&a.ss, &v6, sizeof(v6));
    a.len = sizeof(v6);
    return a;
  }
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  if (getaddrinfo(h.c_str(), nullptr, &hints, &res) != 0 || !res) throw Error("ResolveFailed", h);
  std::memcpy(&a.ss, res->ai_addr, res->ai_addrlen);
  a.len = socklen_t(res->ai_addrlen);
  freeaddrinfo(res);
  if (a.ss.ss_family == AF_INET) reinterpret_cast<sockaddr_in*>(&a.ss)->sin_port = htons(port);
  else reinterpret_cast<sockaddr_in6*>(&a.ss)->sin6_port = htons(port);
  return a;
}

std::optional<Addr> resolve_with_deadline(const std::string& host_port, uint16_t default_port, int timeout_ms) {
  if (const char* m = std::getenv("ZEST_DHT_HOSTS")) {
    const std::string map = m;
    const std::string host = host_port.substr(0, host_port.rfind(':'));
    size_t p = 0;
    while (p <= map.size()) {
      size_t e = map.find(',', p);
      if (e == std::string::npos) e = map.size();
      const std::string item = map.substr(p, e - p);
      const size_t eq = item.find('=');
      if (eq != std::string::npos && (item.substr(0, eq) == host || item.substr(0, eq) == host_port)) {
        try {
          return Addr::parse(item.substr(eq + 1), default_port);
        } catch (const Error&) {
          return std::nullopt;
        }
      }
      p = e + 1;
    }
  }
  struct State {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    std::optional<Addr> addr;
  };
  auto st = std::make_shared<State>();
  // Detached: it owns only `st`, so a resolver that outlives the deadline touches nothing of ours.
  std::thread([st, host_port, default_port] {
    std::optional<Addr> a;
    try {
      a = Addr::parse(host_port, default_port);
    } catch (const Error&) {
    }
    std::lock_guard<std::mutex> g(st->mu);
    st->addr = a;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lk(st->mu);
  st->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return st->done; });
  return st->done ? st->addr : std::nullopt;
}

Addr Addr::ipv4(const uint8_t ip[4], uint16_t port) {
  Addr a;
  sockaddr_in v4{};
  v4.sin_family = AF_INET;
  v4.sin_port = htons(port);
  std::memcpy(&v4.sin_addr, ip, 4);
  std::memcpy(&a.ss, &v4, sizeof(v4));
  a.len = sizeof(v4);
  return a;
}

Addr Addr::any(uint16_t port) {
  const uint8_t z[4] = {0, 0, 0, 0};
  return ipv4(z, port);
}

Addr Addr::loopback(uint16_t port) {
  const uint8_t l[4] = {127, 0, 0, 1};
  return ipv4(l, port);
}

uint16_t Addr::port() const {
  if (ss.ss_family == AF_INET) return ntohs(reinterpret_cast<const sockaddr_in*>(&ss)->sin_port);
  if (ss.ss_family == AF_INET6) return ntohs(reinterpret_cast<const sockaddr_in6*>(&ss)->sin6_port);
  return 0;
}

void Addr::ipv4_bytes(uint8_t out[4]) const {
  std::memcpy(out, &reinterpret_cast<const sockaddr_in*>(&ss)->sin_addr, 4);
}

std::string Addr::host() const {
  char buf[INET6_ADDRSTRLEN] = {0};
  if (ss.ss_family == AF_INET)
    inet_ntop(AF_INET, &reinterpret_cast<const sockaddr_in*>(&ss)->sin_addr, buf, sizeof(buf));
  else if (ss.ss_family == AF_INET6)
    inet_ntop(AF_INET6, &reinterpret_cast<const sockaddr_in6*>(&ss)->sin6_addr, buf, sizeof(buf));
  return buf;
}

std::string Addr::str() const {
  if (ss.ss_family == AF_INET6) return "[" + host() + "]:" + std::to_string(port());
  return host() + ":" + std::to_string(port());
}

bool Addr::operator==(const Addr& o) const {
  if (ss.ss_family != o.ss.ss_family || port() != o.port()) return false;
  if (ss.ss_family == AF_INET)
    return std::memcmp(&reinterpret_cast<const sockaddr_in*>(&ss)->sin_addr,
                       &reinterpret_cast<const sockaddr_in*>(&o.ss)->sin_addr, 4) == 0;
  return std::memcmp(&reinterpret_cast<const sockaddr_in6*>(&ss)->sin6_addr,
                     &reinterpret_cast<const sockaddr_in6*>(&o.ss)->sin6_addr, 16) == 0;
}

Socket& Socket::operator=(Socket&& o) noexcept {
  if (this != &o) {
    close();
    fd_ = o.fd_;
    timeout_ms_ = o.timeout_ms_;
    o.fd_ = -1;
  }
  return *this;
}

Socket Socket::connect_tcp(const Addr& a, int timeout_ms) {
  int fd = ::socket(a.ss.ss_family, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (fd < 0) sys_fail("socket");
  Socket s(fd);
  int r = ::connect(fd, reinterpret_cast<const sockaddr*>(&a.ss), a.len);
  if (r < 0 && errno != EINPROGRESS) throw Error("ConnectFailed", a.str() + ": " + std::strerror(errno));
  if (r < 0) {
    if (!poll_fd(fd, POLLOUT, timeout_ms)) throw Error("Timeout", "connect " + a.str());
    int err = 0;
    socklen_t el = sizeof(err);
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el);
    if (err) throw Error("ConnectFailed", a.str() + ": " + std::strerror(err));
  }
  int flags = fcntl(fd, F_GETFL);
  fcntl(fd, F_SETFL, flags & ~O_NONBLOCK);
  s.set_nodelay();
  return s;
}

Socket Socket::listen_tcp(const Addr& bind_addr, int backlog) {
  int fd = ::socket(bind_addr.ss.ss_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) sys_fail("socket");
  Socket s(fd);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (::bind(fd, reinterpret_cast<const sockaddr*>(&bind_addr.ss), bind_addr.len) < 0)
    throw Error("BindFailed", bind_addr.str() + ": " + std::strerror(errno));
  if (::listen(fd, backlog) < 0) sys_fail("listen");
  return s;
}

Socket Socket::udp(const Addr& bind_addr) {
  int fd = ::socket(bind_addr.ss.ss_family, SOCK_DGRAM | SOCK_CLOEXEC, 0);
  if (fd < 0) sys_fail("socket");
  Socket s(fd);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (::bind(fd, reinterpret_cast<const sockaddr*>(&bind_addr.ss), bind_addr.len) < 0)
    throw Error("BindFailed", bind_addr.str() + ": " + std::strerror(errno));
  return s;
}

Socket Socket::accept(int timeout_ms, Addr* peer) {
  if (!poll_fd(fd_, POLLIN, timeout_ms)) return Socket();
  Addr a;
  a.len = sizeof(a.ss);
  int c = ::accept4(fd_, reinterpret_cast<sockaddr*>(&a.ss), &a.len, SOCK_CLOEXEC);
  if (c < 0) {
    if (errno == EINTR || errno == EAGAIN || errno == ECONNABORTED) return Socket();
    if (errno == EBADF || errno == EINVAL) throw Error("Closed", "listener closed");
    sys_fail("accept");
  }
  if (peer) *peer = a;
  Socket s(c);
  s.set_nodelay();
  return s;
}

void Socket::set_timeout(int ms) { timeout_ms_ = ms; }

void Socket::set_nodelay() {
  int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

void Socket::set_buffers(int bytes) {
  setsockopt(fd_, SOL_SOCKET, SO_SNDBUF, &bytes, sizeof(bytes));
  setsockopt(fd_, SOL_SOCKET, SO_RCVBUF, &bytes, sizeof(bytes));
}

bool Socket::wait_readable(int timeout_ms) const { return poll_fd(fd_, POLLIN, timeout_ms); }

void Socket::write_all(const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  while (n) {
    if (timeout_ms_ > 0 && !poll_fd(fd_, POLLOUT, timeout_ms_)) throw Error("Timeout", "write");
    ssize_t w = ::send(fd_, b, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw Error("WriteFailed", std::strerror(errno));
    }
    b += w;
    n -= size_t(w);
  }
}

void Socket::writev_all(iovec* iov, int n) {
  while (n > 0) {
    if (timeout_ms_ > 0 && !poll_fd(fd_, POLLOUT, timeout_ms_)) throw Error("Timeout", "write");
    msghdr mh{};
    mh.msg_iov = iov;
    mh.msg_iovlen = size_t(n);
    ssize_t w = ::sendmsg(fd_, &mh, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw Error("WriteFailed", std::strerror(errno));
    }
    size_t left = size_t(w);
    while (n > 0 && left >= iov->iov_len) {
      left -= iov->iov_len;
      ++iov;
      --n;
    }
    if (n > 0) {
      iov->iov_base = static_cast<uint8_t*>(iov->iov_base) + left;
      iov->iov_len -= left;
    }
  }
}

size_t Socket::read_some(void* p, size_t n) {
  while (true) {
    if (timeout_ms_ > 0 && !poll_fd(fd_, POLLIN, timeout_ms_)) throw Error("Timeout", "read");
    ssize_t r = ::recv(fd_, p, n, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw Error("ReadFailed", std::strerror(errno));
    }
    return size_t(r);
  }
}

void Socket::read_exact(void* p, size_t n) {
  uint8_t* b = static_cast<uint8_t*>(p);
  while (n) {
    size_t r = read_some(b, n);
    if (r == 0) throw Error("ConnectionClosed");
    b += r;
    n -= r;
  }
}

void Socket::send_to(const Addr& a, const void* p, size_t n) {
  ssize_t w = ::sendto(fd_, p, n, MSG_NOSIGNAL, reinterpret_cast<const sockaddr*>(&a.ss), a.len);
  if (w < 0) throw Error("WriteFailed", std::strerror(errno));
}

size_t Socket::recv_from(void* p, size_t n, Addr* from, int timeout_ms) {
  if (!poll_fd(fd_, POLLIN, timeout_ms)) return 0;
  Addr a;
  a.len = sizeof(a.ss);
  ssize_t r = ::recvfrom(fd_, p, n, 0, reinterpret_cast<sockaddr*>(&a.ss), &a.len);
  if (r < 0) {
    if (errno == EINTR || errno == EAGAIN) return 0;
    throw Error("ReadFailed", std::strerror(errno));
  }
  if (from) *from = a;
  return size_t(r);
}

Addr Socket::local_addr() const {
  Addr a;
  a.len = sizeof(a.ss);
  getsockname(fd_, reinterpret_cast<sockaddr*>(&a.ss), &a.len);
  return a;
}

void Socket::shutdown() {
  if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
}

void Socket::close() {
  if (fd_ >= 0) {
    ::close(fd_);
    fd_ = -1;
  }
}

}  // namespace zest::net
