#!/bin/bash
# Round 3: BASELINE config-2 shape (1 seeder + 1 leecher) and an odd rank count (3), self-launched
# bench.py rehearsals on one GPU (gloo control plane, ranks share the device; not xGMI numbers).
OUT=gpurun_out/r3cfg2; mkdir -p $OUT
export ZEST_SKIP_BUILD=1 ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1
timeout -k 10 400 python -u bench.py --gpus 2 --seeders 1 --model llama-3.1-8b --steps 3 --warmup 1 \
  > $OUT/seed1_leech1.log 2>&1 || { tail -30 $OUT/seed1_leech1.log; exit 1; }
grep -h "^\[bench\] .*aggregate\|^\[bench\] exchange" $OUT/seed1_leech1.log
timeout -k 10 400 python -u bench.py --gpus 3 --model llama-3.1-8b --steps 3 --warmup 1 \
  > $OUT/n3.log 2>&1 || { tail -30 $OUT/n3.log; exit 1; }
grep -h "^\[bench\] .*aggregate\|^\[bench\] exchange" $OUT/n3.log
