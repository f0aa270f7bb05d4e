#!/bin/bash
# GPU box: kernel tests + rocprofv3 kernel-trace/stats of the pull bench (Llama-3.1-8B, 1 GPU).
# Usage (from this container): gpurun --timeout 1100 -- 'bash tools/gpu/gpu_profile.sh'
export ZEST_SKIP_BUILD=1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench8b -- \
  python3 bench.py --model llama-3.1-8b --steps 2 --warmup 1 > gpurun_out/prof_bench8b.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_bench8b.log
if [ $rc -ne 0 ]; then exit $rc; fi
find gpurun_out/prof -name "*stats*.csv" | head -20
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench70b.log 2>&1
echo "bench70b rc=$?"; tail -1 gpurun_out/bench70b.log
