#!/bin/bash
# Round 3: traced GPU CLI pull (where do init and the write tail go?), then the IPC bisect.
OUT=gpurun_out/r3c8; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 600 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --skip-host \
  --out $OUT/cli_sync.json \
  --cli-configs "ZEST_GPU_TRACE=$PWD/$OUT/trace2.json;ZEST_GPU_TRACE=$PWD/$OUT/trace1.json,ZEST_GPU_PIPES=1" \
  > $OUT/cli_sync.log 2>&1 || { tail -30 $OUT/cli_sync.log; exit 1; }
grep -h "^\[" $OUT/cli_sync.log
for t in trace2 trace1; do python tools/trace_summary.py $OUT/$t.json.0 --top 30 > $OUT/$t.txt; cat $OUT/$t.txt; done
bash tools/gpu/gpu_r3_ipc2.sh
