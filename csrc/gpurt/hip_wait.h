// Host waits on HIP events that leave the CPU to others.
//
// hipEventSynchronize polls: a thread waiting for an H2D copy or a batch's kernels keeps a core busy
// for as long as the GPU takes (the streaming pipeline's releaser thread cost 0.18 CPU-s per 0.6 s
// pull, per rank, in the 8-rank rehearsal -- profiles/r6/thread_cpu_r6r/).  These waits are for
// batch-sized work (milliseconds), so a query + short sleeps (backing off to `max_us`) costs a
// sleep's slack of latency and almost no CPU.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <thread>

namespace zest::gpu {

inline hipError_t idle_event_sync(hipEvent_t e, int max_us = 50) {
  hipError_t r = hipEventQuery(e);
  int us = 5;
  while (r == hipErrorNotReady) {
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    us = std::min(us * 2, max_us);
    r = hipEventQuery(e);
  }
  return r;
}

// The same for everything queued on `s` so far (an event recorded behind it).
inline hipError_t idle_stream_sync(hipStream_t s, int max_us = 50) {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return hipStreamSynchronize(s);
  hipError_t r = hipEventRecord(e, s);
  if (r == hipSuccess) r = idle_event_sync(e, max_us);
  (void)hipEventDestroy(e);
  return r;
}

}  // namespace zest::gpu
