#!/bin/bash
# Leaf-flat K1 check: numerics tests (hash + ingest), kernel timings (wave vs flat) on 1 GiB, and
# a kernel trace of the flat pipeline with a device sync between launches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hf
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/hf/tests.log 2>&1 || { tail -40 gpurun_out/hf/tests.log; exit 1; }
tail -3 gpurun_out/hf/tests.log
timeout -k 10 300 python -u tools/kbench.py --gib 1 --iters 5 --only hash,place > gpurun_out/hf/kbench.log 2>&1 || { tail -20 gpurun_out/hf/kbench.log; exit 1; }
cat gpurun_out/hf/kbench.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/hf/kt -o kt -- python3 tools/experiments/hash_plan_probe.py 16384 65536 > gpurun_out/hf/kt.log 2>&1 || exit $?
echo done
