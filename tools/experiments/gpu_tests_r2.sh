#!/bin/bash
# GPU test suite + smoke (round 2); logs under gpurun_out/r2/.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/r2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/r2/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r2/smoke.log
