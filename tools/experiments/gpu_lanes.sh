#!/bin/bash
# Two compute lanes in the device engine: GPU tests, then the 1-GPU bench in random and bf16 modes.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/lanes
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/lanes/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lanes/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/lanes/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/lanes/bench_random.log 2>&1 || exit $?
tail -1 gpurun_out/lanes/bench_random.log | cut -c1-200
timeout -k 10 500 python bench.py --mode bf16 --steps 2 --warmup 1 > gpurun_out/lanes/bench_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/lanes/bench_bf16.log | cut -c1-200
