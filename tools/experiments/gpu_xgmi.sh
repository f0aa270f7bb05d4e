#!/bin/bash
# K8 (xgmi exchange) check: IPC/xgmi GPU tests, then the gather micro-benchmark.
mkdir -p gpurun_out/xgmi
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ipc.py \
    > gpurun_out/xgmi/tests.log 2>&1
rc=$?; tail -8 gpurun_out/xgmi/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/kbench.py --only gather > gpurun_out/xgmi/kbench.log 2>&1
rc=$?; cat gpurun_out/xgmi/kbench.log; exit $rc
