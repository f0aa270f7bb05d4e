#!/bin/bash
export ZEST_SKIP_BUILD=1 ZG_LZ4_PROF=1
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py --only lz4,lz4big --iters 1 > gpurun_out/lz4prof.log 2>&1
rc=$?; echo "rc=$rc"; grep -v "^/opt" gpurun_out/lz4prof.log | tail -30
exit $rc
