#!/bin/bash
# Round 3: data-mode order A/B with the pinned-origin pool, then the GPU test suite.
OUT=gpurun_out/r3modes; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $OUT/bench_bf16_random.log 2>&1 || { tail -30 $OUT/bench_bf16_random.log; exit 1; }
grep -h "aggregate" $OUT/bench_bf16_random.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --modes random,bf16 > $OUT/bench_random_bf16.log 2>&1 || { tail -30 $OUT/bench_random_bf16.log; exit 1; }
grep -h "aggregate" $OUT/bench_random_bf16.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
