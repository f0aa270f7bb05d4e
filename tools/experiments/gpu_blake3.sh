#!/bin/bash
# BLAKE3 hashing check after a kernel change: GPU kernel tests, then the hash micro-benchmark.
set -o pipefail
mkdir -p gpu_out gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py > gpurun_out/blake3_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/kbench.py --only hash > gpurun_out/blake3_kbench.log 2>&1 &&
timeout -k 10 200 python -u tools/kbench.py --only place >> gpurun_out/blake3_kbench.log 2>&1
rc=$?
if [ $rc -eq 0 ] && [ -f gpu_ab/_hip_old.so ]; then
  so=zest_amd/_hip.cpython-310-x86_64-linux-gnu.so
  cp $so /tmp/_hip_new.so && cp gpu_ab/_hip_old.so $so &&
  echo "--- previous kernel" >> gpurun_out/blake3_kbench.log &&
  timeout -k 10 200 python -u tools/kbench.py --only hash >> gpurun_out/blake3_kbench.log 2>&1
  rc=$?
  cp /tmp/_hip_new.so $so
fi
tail -5 gpurun_out/blake3_tests.log; cat gpurun_out/blake3_kbench.log
exit $rc
