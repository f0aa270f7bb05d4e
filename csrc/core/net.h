// Sockets with deadlines (TCP/UDP, IPv4+IPv6) for the BitTorrent, DHT, tracker and HTTP layers.
//
// The reference runs on Zig std.Io with no timeouts anywhere ("no timeouts ... TCP
// reads, DHT receive dht.zig:420, HTTP"); every blocking call here takes a deadline and throws
// Error("Timeout") instead of hanging.
#pragma once

#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/uio.h>

#include <cstdint>
#include <optional>
#include <string>
#include <string_view>

#include "common.h"

namespace zest::net {

struct Addr {
  sockaddr_storage ss{};
  socklen_t len = 0;

  static Addr parse(std::string_view host_port, uint16_t default_port = 0);  // "ip:port", "[v6]:port", "host:port"
  static Addr resolve(std::string_view host, uint16_t port);                 // DNS (getaddrinfo)
  static Addr ipv4(const uint8_t ip[4], uint16_t port);
  static Addr any(uint16_t port);        // 0.0.0.0:port
  static Addr loopback(uint16_t port);   // 127.0.0.1:port
  uint16_t port() const;
  bool is_v4() const { return ss.ss_family == AF_INET; }
  // 4-byte IPv4 address (only valid when is_v4()).
  void ipv4_bytes(uint8_t out[4]) const;
  std::string str() const;
  std::string host() const;
  bool operator==(const Addr& o) const;
  bool operator!=(const Addr& o) const { return !(*this == o); }
};

// Resolve "host:port" with a deadline: a hosts override (ZEST_DHT_HOSTS="name=ip:port,...", for
// air-gapped labs and tests) first, then getaddrinfo on a helper thread (getaddrinfo itself has no
// timeout; an offline resolver can block for many seconds).  nullopt when unresolved in time.
std::optional<Addr> resolve_with_deadline(const std::string& host_port, uint16_t default_port, int timeout_ms);

class Socket {
 public:
  Socket() = default;
  explicit Socket(int fd) : fd_(fd) {}
  Socket(Socket&& o) noexcept : fd_(o.fd_) { o.fd_ = -1; }
  Socket& operator=(Socket&& o) noexcept;
  Socket(const Socket&) = delete;
  Socket& operator=(const Socket&) = delete;
  ~Socket() { close(); }

  static Socket connect_tcp(const Addr& a, int timeout_ms);
  static Socket listen_tcp(const Addr& bind, int backlog = 256);
  static Socket udp(const Addr& bind);

  // Accept with a timeout (ms, -1 = forever); returns an invalid socket on timeout.
  Socket accept(int timeout_ms, Addr* peer = nullptr);
  void set_timeout(int ms);  // per-operation deadline for read/write (0 = none)
  void set_nodelay();
  void set_buffers(int bytes);

  void write_all(const void* p, size_t n);
  void writev_all(iovec* iov, int n);
  void read_exact(void* p, size_t n);
  size_t read_some(void* p, size_t n);  // 0 = orderly close
  // Wait until readable; false on timeout.
  bool wait_readable(int timeout_ms) const;

  // UDP
  void send_to(const Addr& a, const void* p, size_t n);
  // Returns bytes received, 0 on timeout.
  size_t recv_from(void* p, size_t n, Addr* from, int timeout_ms);

  Addr local_addr() const;
  void shutdown();
  void close();
  int fd() const { return fd_; }
  bool valid() const { return fd_ >= 0; }

 private:
  int fd_ = -1;
  int timeout_ms_ = 0;
};

}  // namespace zest::net
