#!/bin/bash
# Round 3: bf16 (BG4-LZ4) 70B pull at N=1 -- pipeline knobs A/B: staging slots and round size.
OUT=gpurun_out/r3shape; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
for cfg in "--slots 4" "--slots 6" "--round-mb 2048" "--round-mb 512"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 400 python -u bench.py --modes bf16 --steps 5 --warmup 2 $cfg > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
  echo "$cfg: $(grep -h 'aggregate' $OUT/$tag.log)"
done
