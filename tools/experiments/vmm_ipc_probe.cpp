// Does sharing HBM between two processes on ONE GPU work through the VMM API (hipMemCreate chunks
// exported as dmabuf fds, passed with SCM_RIGHTS, imported with hipMemImportFromShareableHandle and
// mapped into one contiguous range), where hipIpcOpenMemHandle of a >= 2 GiB allocation hangs?
//
// The parent forks BEFORE any HIP call (a child cannot use HIP after its parent initialised it).
// Exporter: reserves `total` bytes of VA, backs them with `chunk`-sized physical allocations, fills
// chunk k with byte (k & 0xff) (hipMemset), sends the fds.  Importer: imports every fd, maps them
// contiguously, checks the first byte of every chunk with a D2H copy, and times the import.
//
// Build: hipcc -O2 --offload-arch=gfx950 -o vmm_ipc_probe tools/experiments/vmm_ipc_probe.cpp
// Run:   vmm_ipc_probe <total GiB> <chunk MiB> [own] [dup]     (e.g. 16 512)
//   own: the importer first makes (and maps) a VMM arena of its own, as every rank does
//   dup: the exporter sends dup()s of its fds, as the Python server does
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "[%d] %s: %s\n", int(getpid()), #x, hipGetErrorString(e_)); \
      std::exit(3);                                                                   \
    }                                                                                 \
  } while (0)

static void send_fds(int sock, const std::vector<int>& fds) {
  for (size_t i = 0; i < fds.size(); i += 200) {
    const size_t n = std::min<size_t>(200, fds.size() - i);
    char byte = 'f';
    iovec iov{&byte, 1};
    std::vector<char> ctl(CMSG_SPACE(sizeof(int) * n));
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = ctl.data();
    m.msg_controllen = ctl.size();
    cmsghdr* c = CMSG_FIRSTHDR(&m);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(sizeof(int) * n);
    std::memcpy(CMSG_DATA(c), fds.data() + i, sizeof(int) * n);
    if (sendmsg(sock, &m, 0) != 1) std::exit(4);
  }
}

static std::vector<int> recv_fds(int sock, size_t count) {
  std::vector<int> out;
  while (out.size() < count) {
    const size_t n = std::min<size_t>(200, count - out.size());
    char byte;
    iovec iov{&byte, 1};
    std::vector<char> ctl(CMSG_SPACE(sizeof(int) * n));
    msghdr m{};
    m.msg_iov = &iov;
    m.msg_iovlen = 1;
    m.msg_control = ctl.data();
    m.msg_controllen = ctl.size();
    if (recvmsg(sock, &m, 0) != 1) std::exit(5);
    cmsghdr* c = CMSG_FIRSTHDR(&m);
    const size_t got = (c->cmsg_len - CMSG_LEN(0)) / sizeof(int);
    const int* p = reinterpret_cast<const int*>(CMSG_DATA(c));
    out.insert(out.end(), p, p + got);
  }
  return out;
}

static hipMemAllocationProp prop_for(int dev) {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = dev;
  return p;
}

static void on_segv(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "SIGSEGV backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int main(int argc, char** argv) {
  signal(SIGSEGV, on_segv);
  bool own = false, dup_fds = false;
  for (int i = 3; i < argc; ++i) {
    own = own || std::strcmp(argv[i], "own") == 0;
    dup_fds = dup_fds || std::strcmp(argv[i], "dup") == 0;
  }
  const size_t total = size_t(std::atof(argc > 1 ? argv[1] : "16") * double(1ull << 30));
  const size_t chunk = size_t(std::atoi(argc > 2 ? argv[2] : "512")) << 20;
  const size_t n = (total + chunk - 1) / chunk;
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 1;
  const pid_t child = fork();
  if (child < 0) return 1;
  CK(hipSetDevice(0));
  const hipMemAllocationProp prop = prop_for(0);
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  if (chunk % gran) {
    std::fprintf(stderr, "chunk %zu is not a multiple of the granularity %zu\n", chunk, gran);
    return 2;
  }
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, n * chunk, 0, nullptr, 0));
  auto* base = static_cast<uint8_t*>(va);
  if (child > 0) {  // exporter
    close(sv[1]);
    double t0 = now();
    std::vector<hipMemGenericAllocationHandle_t> h(n);
    std::vector<int> fds(n);
    for (size_t k = 0; k < n; ++k) {
      CK(hipMemCreate(&h[k], chunk, &prop, 0));
      CK(hipMemMap(base + k * chunk, chunk, 0, h[k], 0));
      int fd = -1;
      CK(hipMemExportToShareableHandle(&fd, h[k], hipMemHandleTypePosixFileDescriptor, 0));
      fds[k] = fd;
    }
    CK(hipMemSetAccess(base, n * chunk, &acc, 1));
    for (size_t k = 0; k < n; ++k) CK(hipMemset(base + k * chunk, int(k & 0xff), chunk));
    CK(hipDeviceSynchronize());
    std::printf("exporter: %zu x %zu MiB created, mapped, filled, exported (granularity %zu KiB) in %.3f s\n", n,
                chunk >> 20, gran >> 10, now() - t0);
    std::fflush(stdout);
    if (dup_fds)
      for (auto& fd : fds) fd = dup(fd);
    send_fds(sv[0], fds);
    char done = 0;
    if (read(sv[0], &done, 1) != 1) done = 'x';
    int st = 0;
    waitpid(child, &st, 0);
    std::printf("exporter: importer exited %d, said '%c'\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1, done);
    return WIFEXITED(st) && WEXITSTATUS(st) == 0 && done == 'k' ? 0 : 1;
  }
  // importer
  close(sv[0]);
  if (own) {  // an arena of the importer's own, mapped in its own range
    void* ova = nullptr;
    CK(hipMemAddressReserve(&ova, n * chunk, 0, nullptr, 0));
    for (size_t k = 0; k < n; ++k) {
      hipMemGenericAllocationHandle_t h;
      CK(hipMemCreate(&h, chunk, &prop, 0));
      CK(hipMemMap(static_cast<uint8_t*>(ova) + k * chunk, chunk, 0, h, 0));
    }
    CK(hipMemSetAccess(ova, n * chunk, &acc, 1));
    std::printf("importer: own arena of %zu chunks mapped\n", n);
    std::fflush(stdout);
  }
  const std::vector<int> fds = recv_fds(sv[1], n);
  double t0 = now();
  for (size_t k = 0; k < n; ++k) {
    hipMemGenericAllocationHandle_t h;
    CK(hipMemImportFromShareableHandle(&h, reinterpret_cast<void*>(static_cast<intptr_t>(fds[k])),
                                       hipMemHandleTypePosixFileDescriptor));
    CK(hipMemMap(base + k * chunk, chunk, 0, h, 0));
    close(fds[k]);
  }
  CK(hipMemSetAccess(base, n * chunk, &acc, 1));
  const double t_imp = now() - t0;
  int bad = 0;
  for (size_t k = 0; k < n; ++k) {
    uint8_t b = 0;
    CK(hipMemcpy(&b, base + k * chunk + chunk - 1, 1, hipMemcpyDeviceToHost));
    if (b != uint8_t(k & 0xff)) ++bad;
  }
  std::printf("importer: %zu chunks (%.1f GiB) imported + mapped in %.3f s, %d bad\n", n,
              double(n * chunk) / double(1ull << 30), t_imp, bad);
  std::fflush(stdout);
  const char ok = bad ? 'b' : 'k';
  if (write(sv[1], &ok, 1) != 1) return 6;
  return bad ? 1 : 0;
}
