#!/bin/bash
# Round checkpoint on the GPU box: all GPU tests, smoke(), host synthetic bench, 70B bench + profile.
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/gpu_tests_all.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
./zest_amd/_bin/zest bench --synthetic > gpurun_out/host_bench.txt 2>&1; cat gpurun_out/host_bench.txt
lscpu | grep -E "Model name|MHz" > gpurun_out/host_cpu.txt 2>/dev/null; cat gpurun_out/host_cpu.txt
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench70b.log 2>&1
rc=$?; echo "bench70b rc=$rc"; tail -1 gpurun_out/bench70b.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench70b -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_bench70b.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
