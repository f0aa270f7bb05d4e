// Host-memory probe for the GPU worker's write-back (host calls only; no kernels):
//  * what does pinning 1 GiB cost: hipHostMalloc vs mmap (+ MADV_HUGEPAGE) + hipHostRegister?
//  * how fast does pwrite read from each kind of buffer (the page-cache copy reads the source)?
//  * D2H of 64 MiB into each.
// Build: hipcc -O2 --offload-arch=gfx950 -o build/experiments/pinned_probe tools/experiments/pinned_probe.cpp
// Run:   pinned_probe <dir>   (writes and deletes <dir>/pinned_probe.bin)
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

static const size_t kBytes = size_t(1) << 30, kPiece = size_t(64) << 20;

static double pwrite_rate(const std::string& path, const uint8_t* src) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return -1;
  const double t0 = now();
  for (size_t off = 0; off < kBytes; off += kPiece) {
    size_t done = 0;
    while (done < kPiece) {
      const ssize_t w = ::pwrite(fd, src + off + done, kPiece - done, off_t(off + done));
      if (w <= 0) return -1;
      done += size_t(w);
    }
  }
  const double dt = now() - t0;
  ::close(fd);
  ::unlink(path.c_str());
  return kBytes / dt / 1e9;
}

static double d2h_rate(uint8_t* host, const uint8_t* dev, hipStream_t s) {
  CK(hipMemcpyAsync(host, dev, kPiece, hipMemcpyDeviceToHost, s));  // warm
  CK(hipStreamSynchronize(s));
  const double t0 = now();
  for (size_t off = 0; off < kBytes; off += kPiece) CK(hipMemcpyAsync(host + off, dev + off, kPiece, hipMemcpyDeviceToHost, s));
  CK(hipStreamSynchronize(s));
  return kBytes / (now() - t0) / 1e9;
}

int main(int argc, char** argv) {
  const std::string path = std::string(argc > 1 ? argv[1] : "/tmp") + "/pinned_probe.bin";
  double t0 = now();
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  std::printf("hip init %.1f ms\n", (now() - t0) * 1e3);
  uint8_t* dev = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&dev), kBytes));
  CK(hipMemset(dev, 7, kBytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  // 1. hipHostMalloc (default flags), and with hipHostMallocNonCoherent
  const unsigned flags[2] = {hipHostMallocDefault, hipHostMallocNonCoherent};
  const char* names[2] = {"hipHostMalloc default", "hipHostMalloc noncoherent"};
  for (int k = 0; k < 2; ++k) {
    uint8_t* h = nullptr;
    t0 = now();
    CK(hipHostMalloc(reinterpret_cast<void**>(&h), kBytes, flags[k]));
    const double alloc = now() - t0;
    t0 = now();
    std::memset(h, 1, kBytes);
    const double touch = now() - t0;
    const double d2h = d2h_rate(h, dev, s);
    const double pw = pwrite_rate(path, h);
    std::printf("%-28s alloc %7.1f ms  first touch %6.1f ms  D2H %6.1f GB/s  pwrite from it %6.2f GB/s\n", names[k],
                alloc * 1e3, touch * 1e3, d2h, pw);
    t0 = now();
    CK(hipHostFree(h));
    std::printf("%-28s free %.1f ms\n", names[k], (now() - t0) * 1e3);
  }
  // 2. mmap (+ THP advice) + populate + hipHostRegister
  for (int huge = 0; huge < 2; ++huge) {
    t0 = now();
    void* m = mmap(nullptr, kBytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) return 1;
    if (huge) madvise(m, kBytes, MADV_HUGEPAGE);
    std::memset(m, 1, kBytes);
    const double touch = now() - t0;
    t0 = now();
    CK(hipHostRegister(m, kBytes, hipHostRegisterDefault));
    const double reg = now() - t0;
    auto* h = static_cast<uint8_t*>(m);
    const double d2h = d2h_rate(h, dev, s);
    const double pw = pwrite_rate(path, h);
    std::printf("%-28s mmap+touch %6.1f ms  register %7.1f ms  D2H %6.1f GB/s  pwrite from it %6.2f GB/s\n",
                huge ? "mmap THP + hipHostRegister" : "mmap 4K + hipHostRegister", touch * 1e3, reg * 1e3, d2h, pw);
    t0 = now();
    CK(hipHostUnregister(m));
    munmap(m, kBytes);
    std::printf("%-28s unregister+unmap %.1f ms\n", huge ? "mmap THP" : "mmap 4K", (now() - t0) * 1e3);
  }
  // 3. plain pageable memory (reference pwrite rate)
  {
    auto* h = static_cast<uint8_t*>(std::malloc(kBytes));
    std::memset(h, 1, kBytes);
    std::printf("%-28s pwrite from it %6.2f GB/s\n", "malloc (pageable)", pwrite_rate(path, h));
    std::free(h);
  }
  CK(hipFree(dev));
  return 0;
}
