#!/bin/bash
# LZ4 decoder comparison on the GPU: kernel tests (both decoders), then kbench rows for the
# wave-per-chunk (K3b) and thread-per-chunk (K3c) decoders, then the lane ring-size variant.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/kbench.py --only lz4,lz4big,lz4paths > gpurun_out/kbench_lz4_lane.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v "^/opt" gpurun_out/kbench_lz4_lane.log
if [ $rc -ne 0 ]; then exit $rc; fi
ZG_LZ4_LANE_RING=1024 timeout -k 10 300 python tools/kbench.py --only lz4 > gpurun_out/kbench_lz4_lane1k.log 2>&1
rc=$?; echo "kbench ring1k rc=$rc"; grep -v "^/opt" gpurun_out/kbench_lz4_lane1k.log
exit $rc
