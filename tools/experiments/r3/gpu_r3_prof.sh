#!/bin/bash
# Round 3: GPU CLI pull (native worker, concurrent write-back) vs host pull; 1 vs 3 seeders; rocprofv3
# kernel trace of the 70B bench (bf16 + random modes, fused ingest) -> per-kernel summary.
OUT=gpurun_out/r3p; mkdir -p $OUT
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 600 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --out $OUT/cli_vs_host_8b.json > $OUT/cli_vs_host.log 2>&1 || { tail -30 $OUT/cli_vs_host.log; exit 1; }
grep -h "^\[" $OUT/cli_vs_host.log
timeout -k 10 600 python -u tools/stripe_bench.py --mb 4096 --out $OUT/stripe.json > $OUT/stripe.log 2>&1 || { tail -30 $OUT/stripe.log; exit 1; }
grep -h "^\[" $OUT/stripe.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o b70 -- \
  python3 bench.py --steps 3 --warmup 1 > $OUT/prof_bench.log 2>&1 || { tail -30 $OUT/prof_bench.log; exit 1; }
grep -h "aggregate" $OUT/prof_bench.log
DB=$(find $OUT/prof -name "*.db" | head -1)
python tools/rocpd_summary.py "$DB" --title "70B bench, bf16 then random, fused ingest (round 3)" > $OUT/b70_kernels.md 2>&1
head -30 $OUT/b70_kernels.md
rm -f "$DB"
ZEST_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 4 --model llama-3.1-8b --steps 2 --warmup 1 > $OUT/bench_n4_gloo.log 2>&1 || { tail -40 $OUT/bench_n4_gloo.log; exit 1; }
grep -h "aggregate" $OUT/bench_n4_gloo.log
