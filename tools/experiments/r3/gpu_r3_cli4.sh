#!/bin/bash
# Round 3: GPU CLI pull with the worker's parallel init + timeline, vs host pull (sync before each),
# the CLI GPU tests, then the HIP IPC probes (last: a hang there ends the script).
OUT=gpurun_out/r3c4; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 600 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --host-after \
  --out $OUT/cli_sync.json --cli-configs ";ZEST_GPU_WRITERS=4;" \
  > $OUT/cli_sync.log 2>&1 || { tail -30 $OUT/cli_sync.log; exit 1; }
grep -h "^\[" $OUT/cli_sync.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_device.py -k cli \
  > $OUT/cli_tests.log 2>&1 || { tail -30 $OUT/cli_tests.log; exit 1; }
tail -3 $OUT/cli_tests.log
bash tools/gpu/gpu_r3_ipc.sh
