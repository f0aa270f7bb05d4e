// Page-locked host buffers for DMA staging.
//
// Anonymous mmap advised to transparent huge pages, faulted in, then registered with HIP.  Pinning
// 1 GiB this way took 72 ms on the MI355X box against 191 ms for hipHostMalloc (and freeing it 48
// vs 105 ms), with the same 56.5 GB/s D2H and the same pwrite rate from it
// (profiles/pinned_probe_r3.txt): a process that pins a few GiB of staging at start-up -- the
// `zest pull --gpus N` worker -- starts that much sooner.  Falls back to hipHostMalloc when the
// registration is refused.
#pragma once

#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <utility>
#include <vector>

namespace zest::gpurt {

// Touch every page of [p, p + len) so the kernel allocates (and zeroes) it now, from several
// threads for big buffers: one thread faults ~10 GB/s, and a 141 GB pinned origin took tens of
// seconds of bench setup that way.
inline void fault_in(void* p, size_t len) {
  auto* b = static_cast<volatile uint8_t*>(p);
  const size_t per = size_t(1) << 30;
  const size_t nt = std::min<size_t>(16, (len + per - 1) / per);
  auto touch = [b](size_t lo, size_t hi) {
    for (size_t o = lo; o < hi; o += 4096) b[o] = 0;
  };
  if (nt <= 1) {
    touch(0, len);
    return;
  }
  std::vector<std::thread> ts;
  const size_t step = (len / nt + 4095) / 4096 * 4096;
  for (size_t t = 0; t < nt; ++t) {
    const size_t lo = t * step, hi = std::min(len, lo + step);
    if (lo < hi) ts.emplace_back(touch, lo, hi);
  }
  for (auto& t : ts) t.join();
}

class PinnedBuf {
 public:
  PinnedBuf() = default;
  explicit PinnedBuf(size_t n) { alloc(n); }
  ~PinnedBuf() { reset(); }
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  PinnedBuf(PinnedBuf&& o) noexcept { *this = std::move(o); }
  PinnedBuf& operator=(PinnedBuf&& o) noexcept {
    if (this != &o) {
      reset();
      std::swap(p_, o.p_);
      std::swap(n_, o.n_);
      std::swap(mapped_, o.mapped_);
    }
    return *this;
  }

  uint8_t* data() const { return p_; }
  size_t size() const { return n_; }
  // Hand the allocation over to the caller (freed later with free_raw(ptr, size(), mapped())).
  bool mapped() const { return mapped_; }
  uint8_t* release() {
    uint8_t* p = p_;
    p_ = nullptr;
    n_ = 0;
    return p;
  }
  static void free_raw(uint8_t* p, size_t n, bool mapped) {
    if (!p) return;
    if (mapped) {
      (void)hipHostUnregister(p);
      ::munmap(p, n);
    } else {
      (void)hipHostFree(p);
    }
  }

  // Returns false (and holds nothing) when neither path could pin `n` bytes.
  bool alloc(size_t n) {
    reset();
    if (n == 0) n = 1;
    const size_t huge = size_t(2) << 20;
    const size_t len = (n + huge - 1) / huge * huge;
    void* m = ::mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m != MAP_FAILED) {
      (void)::madvise(m, len, MADV_HUGEPAGE);
      fault_in(m, len);  // (2 MiB at a time with THP)
      if (hipHostRegister(m, len, hipHostRegisterDefault) == hipSuccess) {
        p_ = static_cast<uint8_t*>(m);
        n_ = len;
        mapped_ = true;
        return true;
      }
      ::munmap(m, len);
    }
    void* h = nullptr;
    if (hipHostMalloc(&h, n, hipHostMallocDefault) != hipSuccess) return false;
    p_ = static_cast<uint8_t*>(h);
    n_ = n;
    mapped_ = false;
    return true;
  }

  void reset() {
    if (!p_) return;
    if (mapped_) {
      (void)hipHostUnregister(p_);
      ::munmap(p_, n_);
    } else {
      (void)hipHostFree(p_);
    }
    p_ = nullptr;
    n_ = 0;
  }

 private:
  uint8_t* p_ = nullptr;
  size_t n_ = 0;
  bool mapped_ = false;
};

}  // namespace zest::gpurt
