#!/bin/bash
# Device-direct pull vs host pull + GPU load, Llama-3.1-8B from an HBM seeder (tools/direct_bench.py),
# after the direct-pull GPU tests.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_device.py -q -m gpu -x -k "direct or pull_files or cli_pull_gpus" > gpurun_out/gpu_direct_tests.log 2>&1
rc=$?; echo "direct tests rc=$rc"; tail -3 gpurun_out/gpu_direct_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_direct_tests.log | head -20; exit $rc; fi
timeout -k 10 900 python tools/direct_bench.py --model llama-3.1-8b --out gpurun_out/direct_8b.json > gpurun_out/direct_8b.log 2>&1
rc=$?; echo "direct_bench rc=$rc"; grep -v "^/opt" gpurun_out/direct_8b.log | tail -20
exit $rc
