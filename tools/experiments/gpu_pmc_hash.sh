#!/bin/bash
# PMC passes over the BLAKE3 chunk hash and K8 gather kernels (one counter group per run).
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/pmch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K="python3 tools/kbench.py --only hash,gather --iters 1 --gib 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/pmch/p1 -o p1 -- $K > gpurun_out/pmch/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmch/p2 -o p2 -- $K > gpurun_out/pmch/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmch/p3 -o p3 -- $K > gpurun_out/pmch/p3.log 2>&1 || exit $?
echo done
