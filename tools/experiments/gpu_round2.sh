#!/bin/bash
# Round check + evidence: GPU tests, smoke(), 1-GPU bench (random = headline, bf16 = LZ4/BG4 path),
# and a rocprofv3 kernel-trace of the headline bench.
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/round2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/round2/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/round2/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round2/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/round2/smoke.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/round2/bench_n1.log 2>&1 || exit $?
tail -1 gpurun_out/round2/bench_n1.log | cut -c1-200
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --mode bf16 > gpurun_out/round2/bench_n1_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/round2/bench_n1_bf16.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/round2/prof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/round2/prof.log 2>&1 || exit $?
echo profiled
