#!/bin/bash
# Round 3: disk write strategies on the box (host only), then `zest pull --gpus 1` vs host pull with
# `sync` before every timed pull (no dirty pages of an earlier run being flushed under the next one).
OUT=gpurun_out/r3c3; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
df -h /tmp . > $OUT/df.txt 2>&1; mount | grep -E " / | /tmp " >> $OUT/df.txt 2>&1; cat $OUT/df.txt
timeout -k 10 300 python -u tools/experiments/write_probe.py --gb 16 --out $OUT/write_probe.jsonl \
  > $OUT/write_probe.log 2>&1 || { tail -20 $OUT/write_probe.log; exit 1; }
cat $OUT/write_probe.log
timeout -k 10 900 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --host-after \
  --out $OUT/cli_sync.json \
  --cli-configs ";ZEST_GPU_WRITERS=1;ZEST_GPU_WRITERS=4;ZEST_GPU_ODIRECT=1,ZEST_GPU_WRITERS=4,ZEST_GPU_WRITE_SLOTS=2" \
  > $OUT/cli_sync.log 2>&1 || { tail -30 $OUT/cli_sync.log; exit 1; }
grep -h "^\[" $OUT/cli_sync.log
