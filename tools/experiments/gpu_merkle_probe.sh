#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/mkp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mkp/kt -o kt -- python3 tools/experiments/merkle_probe.py > gpurun_out/mkp/kt.log 2>&1 || exit $?
echo done
