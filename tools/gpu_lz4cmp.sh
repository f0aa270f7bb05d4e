#!/bin/bash
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/kbench.py --only lz4,lz4paths > gpurun_out/kbench_lz4_v3.log 2>&1
rc=$?; echo "kbench v3 rc=$rc"; grep -v "^/opt" gpurun_out/kbench_lz4_v3.log
if [ $rc -ne 0 ]; then exit $rc; fi
ZG_LZ4_V2=1 timeout -k 10 300 python tools/kbench.py --only lz4 > gpurun_out/kbench_lz4_v2.log 2>&1
rc=$?; echo "kbench v2 rc=$rc"; grep -v "^/opt" gpurun_out/kbench_lz4_v2.log
exit $rc
