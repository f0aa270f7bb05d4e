#!/bin/bash
# LZ4/BG4 decode diagnosis on one MI355X: cycle profile (ZG_LZ4_PROF), occupancy sweep (ZG_LZ4_GRID
# = persistent-grid cap; 256 blocks = one wave per SIMD) and a PMC pass (instructions, LDS, waits).
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/lz4diag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ZG_LZ4_PROF=1 timeout -k 10 200 python tools/kbench.py --only lz4,lz4paths --iters 1 > gpurun_out/lz4diag/prof.log 2>&1 || exit $?
for g in 256 512 1280; do
  ZG_LZ4_GRID=$g timeout -k 10 200 python tools/kbench.py --only lz4 --iters 3 > gpurun_out/lz4diag/grid$g.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/lz4diag/pmc1 -o pmc1 -- python3 tools/kbench.py --only lz4 --iters 1 > gpurun_out/lz4diag/pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/lz4diag/pmc2 -o pmc2 -- python3 tools/kbench.py --only lz4 --iters 1 > gpurun_out/lz4diag/pmc2.log 2>&1 || exit $?
grep -h "lz4_prof\|ingest_" gpurun_out/lz4diag/*.log | cut -c1-300
