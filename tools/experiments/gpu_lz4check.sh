#!/bin/bash
# LZ4 decoder change check: GPU kernel tests (bit-exact vs host oracle), then decode throughput.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_device.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lz4check_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lz4check_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/lz4check_tests.log | head -20; exit $rc; }
timeout -k 10 300 python tools/kbench.py --only lz4,lz4paths,lz4big --iters 3 > gpurun_out/lz4check_kbench.log 2>&1 || exit $?
ZG_LZ4_PROF=1 timeout -k 10 200 python tools/kbench.py --only lz4 --iters 1 > gpurun_out/lz4check_prof.log 2>&1 || exit $?
grep -h "ingest_\|lz4_prof" gpurun_out/lz4check_kbench.log gpurun_out/lz4check_prof.log | cut -c1-260
