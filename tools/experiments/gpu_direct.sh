#!/bin/bash
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_device.py tests/test_gpu_seed.py -q -m gpu -x > gpurun_out/gpu_direct.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_direct.log
exit $rc
