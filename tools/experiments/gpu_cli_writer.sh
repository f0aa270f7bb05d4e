#!/bin/bash
# zest pull --gpus 1 snapshot-writer A/B (Llama-3.1-8B from an HBM seeder on loopback) + the writer's GPU tests.
# SIMPLE=1 also runs the old writer (one pageable .cpu() copy + one write) for comparison.
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-writer}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_device.py -v -m gpu -x -k "write_device_file or cli_pull_gpus" \
    --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
if [ -n "$SIMPLE" ]; then
  ZEST_GPU_WRITER=simple timeout -k 10 400 python -u tools/direct_bench.py --skip-host --out $OUT/simple.json \
      > $OUT/simple.log 2>&1 || { tail -30 $OUT/simple.log; exit 1; }
  grep "^\[" $OUT/simple.log
fi
timeout -k 10 400 python -u tools/direct_bench.py --skip-host --out $OUT/pipelined.json > $OUT/pipelined.log 2>&1 \
    || { tail -30 $OUT/pipelined.log; exit 1; }
grep "^\[" $OUT/pipelined.log
