#!/bin/bash
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o lz4 -- python3 tools/kbench.py --only lz4 --iters 3 > gpurun_out/prof_lz4.log 2>&1
rc=$?; echo "rc=$rc"; grep kernel gpurun_out/prof_lz4.log | tail -3
exit $rc
