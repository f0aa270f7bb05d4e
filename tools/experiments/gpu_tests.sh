#!/bin/bash
# GPU box: full GPU test suite (one process).
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
exit $rc
