#!/bin/bash
# Round 3: default `--exchange auto` (peer-mapped VMM arenas included) in the self-launched 2-rank
# rehearsal (gloo, ranks share the GPU), both data modes; GPU IPC tests first.
OUT=gpurun_out/r3vmm6; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ipc.py \
  > $OUT/ipc_tests.log 2>&1 || { tail -40 $OUT/ipc_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $OUT/ipc_tests.log
ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 timeout -k 10 600 python bench.py --gpus 2 --model llama-3.1-8b \
  --steps 3 --warmup 1 > $OUT/bench_auto_n2.log 2>&1 || { grep -v amdgpu.ids $OUT/bench_auto_n2.log | tail -60; exit 1; }
grep -h "mapped\|autotune\|GB/s aggregate" $OUT/bench_auto_n2.log | head -12
tail -1 $OUT/bench_auto_n2.log | cut -c1-900
