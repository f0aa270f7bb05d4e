#!/bin/bash
# Kernel trace + one SQ counter pass over the K1 paths (kbench --only hash, 1 GiB).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hfp
K="python3 tools/kbench.py --only hash --iters 2 --gib 1"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/hfp/kt -o kt -- $K > gpurun_out/hfp/kt.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/hfp/p1 -o p1 --output-format csv -- $K > gpurun_out/hfp/p1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/hfp/p2 -o p2 --output-format csv -- $K > gpurun_out/hfp/p2.log 2>&1 || exit $?
find gpurun_out/hfp -name "*stats*" | head; echo done
