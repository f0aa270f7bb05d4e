#!/bin/bash
# GPU tests (incl. 2-rank IPC) + 1-GPU bench after engine changes.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/q2
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/q2/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q2/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/q2/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/q2/bench_n1.log 2>&1 || exit $?
tail -1 gpurun_out/q2/bench_n1.log | cut -c1-220
