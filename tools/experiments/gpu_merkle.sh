#!/bin/bash
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py --only merkle --gib 1 > gpurun_out/kbench_misc.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v "^/opt" gpurun_out/kbench_misc.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --model llama-3.1-8b --steps 3 --warmup 1 > gpurun_out/bench8b.log 2>&1
rc=$?; echo "bench8b rc=$rc"; tail -1 gpurun_out/bench8b.log
exit $rc
