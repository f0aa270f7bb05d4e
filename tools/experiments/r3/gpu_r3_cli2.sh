#!/bin/bash
# Round 3: `zest pull --gpus 1` write-back sweep (writer threads x pinned slots, write-after) vs host
# pull, Llama-3.1-8B from an HBM seeder; host synthetic micro-bench rows on the box's CPU.
OUT=gpurun_out/r3c2; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
./zest_amd/_bin/zest bench --synthetic > $OUT/host_synthetic.txt 2>&1 || exit 1
lscpu | grep -E "Model name|^CPU\(s\)" >> $OUT/host_synthetic.txt
cat $OUT/host_synthetic.txt | head -12
timeout -k 10 900 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --out $OUT/cli_sweep.json \
  --cli-configs "ZEST_GPU_WRITERS=1,ZEST_GPU_WRITE_SLOTS=3;ZEST_GPU_WRITERS=2,ZEST_GPU_WRITE_SLOTS=3;ZEST_GPU_WRITERS=4,ZEST_GPU_WRITE_SLOTS=2;ZEST_GPU_WRITE_AFTER=1,ZEST_GPU_WRITERS=4;ZEST_GPU_ODIRECT=1,ZEST_GPU_WRITERS=4,ZEST_GPU_WRITE_SLOTS=2;ZEST_GPU_ODIRECT=1,ZEST_GPU_WRITE_AFTER=1,ZEST_GPU_WRITERS=4" \
  > $OUT/cli_sweep.log 2>&1 || { tail -30 $OUT/cli_sweep.log; exit 1; }
grep -h "^\[" $OUT/cli_sweep.log
