#!/bin/bash
# Round 3: one-file write concurrency on the box; GPU CLI pull with several device pipelines
# (ZEST_GPU_PIPES) feeding the streaming write-back, vs the host pull (sync before each).
OUT=gpurun_out/r3c7; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 200 python -u tools/experiments/write_probe.py --gb 16 --cases one1,one4,file4 --out $OUT/write_probe.jsonl \
  > $OUT/write_probe.log 2>&1 || { tail -20 $OUT/write_probe.log; exit 1; }
cat $OUT/write_probe.log
timeout -k 10 600 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --host-after \
  --out $OUT/cli_sync.json \
  --cli-configs ";ZEST_GPU_PIPES=1;ZEST_GPU_PIPES=4;ZEST_GPU_PIPES=4,ZEST_GPU_WRITERS=8;" \
  > $OUT/cli_sync.log 2>&1 || { tail -30 $OUT/cli_sync.log; exit 1; }
grep -h "^\[" $OUT/cli_sync.log
