#!/bin/bash
# Round 3: GPU CLI pull (pre-allocated writers, 64 MiB pieces, fast exit) with staging sizes, vs the
# host pull (sync before each); then the HIP IPC probes (last: a hang there ends the script).
OUT=gpurun_out/r3c5; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 600 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --host-after \
  --out $OUT/cli_sync.json \
  --cli-configs ";ZEST_GPU_STAGING_MB=512;ZEST_GPU_STAGING_MB=256;ZEST_GPU_WRITERS=4;ZEST_GPU_PIECE_MB=256;" \
  > $OUT/cli_sync.log 2>&1 || { tail -30 $OUT/cli_sync.log; exit 1; }
grep -h "^\[" $OUT/cli_sync.log
bash tools/gpu/gpu_r3_ipc.sh
