#!/bin/bash
# Host `zest pull` (CPU decode + verify, HF-cache writes) of Llama-3.1-8B from the HBM seeder, traced.
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-host_trace}
mkdir -p $OUT
timeout -k 10 500 python -u tools/direct_bench.py --skip-direct --skip-gpu-cli --trace-host $PWD/$OUT/host.json \
    --out $OUT/host.json.res > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep "^\[" $OUT/bench.log
python tools/trace_summary.py $OUT/host.json > $OUT/summary.txt && cat $OUT/summary.txt
df -h /tmp . | tail -2; nproc; cat /proc/loadavg
rm -f $OUT/host.json
