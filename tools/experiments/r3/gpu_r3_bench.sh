#!/bin/bash
# Round 3: headline bench at N=1 (bf16 headline + random extra) and the self-launched 2-rank
# rehearsal on one GPU (gloo control plane; ranks share the device).
OUT=gpurun_out/r3bench; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 700 python -u bench.py --steps 5 --warmup 2 > $OUT/bench_n1.log 2>&1 || { tail -30 $OUT/bench_n1.log; exit 1; }
tail -3 $OUT/bench_n1.log
ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 timeout -k 10 500 python -u bench.py --gpus 2 --model llama-3.1-8b \
   --steps 2 --warmup 1 > $OUT/bench_n2_gloo.log 2>&1 || { tail -40 $OUT/bench_n2_gloo.log; exit 1; }
tail -2 $OUT/bench_n2_gloo.log
