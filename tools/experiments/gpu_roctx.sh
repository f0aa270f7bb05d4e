#!/bin/bash
# bench.py (1 GPU) with roctx ranges per engine round (ZEST_ROCTX=1) under
# rocprofv3 --marker-trace --kernel-trace.
export ZEST_SKIP_BUILD=1 ZEST_ROCTX=1
mkdir -p gpurun_out/roctx
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace -d gpurun_out/roctx -o bench -- python3 bench.py --steps 1 --warmup 1 --model llama-3.1-8b > gpurun_out/roctx/run.log 2>&1
rc=$?; grep -v "^\s*@" gpurun_out/roctx/run.log | tail -4; exit $rc
