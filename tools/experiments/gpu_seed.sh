#!/bin/bash
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_seed.py tests/test_gpu_device.py -q -m gpu -x > gpurun_out/gpu_seed_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_seed_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/seed_bench.py --model mixtral-8x7b --clients 16 --seconds 20 > gpurun_out/seed_bench.log 2>&1
rc=$?; echo "seed bench rc=$rc"; tail -3 gpurun_out/seed_bench.log
exit $rc
