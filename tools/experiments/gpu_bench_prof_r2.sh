#!/bin/bash
# rocprofv3 kernel trace + stats of the headline bench (Llama-3.1-70B, 1 GPU, random bytes).
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/bprof
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o b70 -- \
  python3 bench.py --steps 3 --warmup 1 > gpurun_out/bprof/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/bprof/bench.log | cut -c1-200
exit $rc
