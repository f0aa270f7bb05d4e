#!/bin/bash
# Round 3: GPU CLI pull with THP-registered pinned staging, 4 device pipelines (default) vs 2, vs
# the host pull (sync before each); one traced run.
OUT=gpurun_out/r3c9; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 600 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --host-after \
  --out $OUT/cli_sync.json \
  --cli-configs ";ZEST_GPU_PIPES=2;ZEST_GPU_TRACE=$PWD/$OUT/trace4.json;" \
  > $OUT/cli_sync.log 2>&1 || { tail -30 $OUT/cli_sync.log; exit 1; }
grep -h "^\[" $OUT/cli_sync.log
python tools/trace_summary.py $OUT/trace4.json.0 --top 30 > $OUT/trace4.txt; cat $OUT/trace4.txt
# VMM-based sharing of HBM between two processes on the one GPU (stop at the first failure)
hipcc -O2 --offload-arch=gfx950 -o $OUT/vmm_ipc_probe tools/experiments/vmm_ipc_probe.cpp || exit 1
for cfg in "2 512" "16 512" "16 2048"; do
  timeout -k 5 60 $OUT/vmm_ipc_probe $cfg > $OUT/vmm_$(echo $cfg | tr ' ' _).txt 2>&1
  rc=$?; echo "vmm [$cfg] rc=$rc"; cat $OUT/vmm_$(echo $cfg | tr ' ' _).txt
  if [ $rc -ne 0 ]; then break; fi
done
rm -f $OUT/vmm_ipc_probe
