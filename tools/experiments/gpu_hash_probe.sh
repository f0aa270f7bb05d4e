#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hpp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/hpp/kt -o kt -- python3 tools/experiments/hash_plan_probe.py 16384 65536 > gpurun_out/hpp/kt.log 2>&1 || exit $?
echo done
