#!/bin/bash
# Round check on the GPU box: full GPU test suite, smoke(), a short 1-GPU bench.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_n1.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_n1.log
exit $rc
