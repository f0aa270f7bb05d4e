#!/bin/bash
# Round 3: peer-mapped exchanges over HIP VMM arenas (dmabuf fds): the GPU IPC tests, then the
# 2-rank bench rehearsal (Llama-3.1-8B, gloo, ranks share the GPU) with --exchange ipc / xgmi / auto.
OUT=gpurun_out/r3vmm; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ipc.py \
  > $OUT/ipc_tests.log 2>&1 || { tail -40 $OUT/ipc_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $OUT/ipc_tests.log
export ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 ZEST_BENCH_WATCHDOG=150 ZEST_EXCHANGE_IPC=1
for ex in xgmi ipc auto; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29561 bench.py --gpus 2 --model llama-3.1-8b --exchange $ex --steps 2 --warmup 1 --modes random \
      > $OUT/bench_$ex.log 2>&1 || { grep -v amdgpu.ids $OUT/bench_$ex.log | tail -60; exit 1; }
  grep -h "mapped\|autotune\|exchange" $OUT/bench_$ex.log | head -6
  tail -1 $OUT/bench_$ex.log | cut -c1-600
done
