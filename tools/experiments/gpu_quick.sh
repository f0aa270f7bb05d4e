#!/bin/bash
# GPU box: kernel tests + LZ4/BG4 ingest microbench.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_device.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py --only lz4,lz4paths ${KB_ARGS} > gpurun_out/kbench_lz4.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kbench_lz4.log | tail -5
exit $rc
