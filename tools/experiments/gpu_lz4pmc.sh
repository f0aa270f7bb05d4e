#!/bin/bash
# PMC passes over the LZ4 decoders (kbench lz4 rows: 256 MiB bf16 LZ4/BG4), one rocprofv3 run per
# counter group.  ZG_LZ4_SEQ=0 in the environment profiles the LDS-ring decoder instead.
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-lz4pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/kbench.py --only lz4 --iters 1 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
echo done
