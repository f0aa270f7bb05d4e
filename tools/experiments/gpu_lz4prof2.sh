#!/bin/bash
# Per-kernel times of the LZ4 decoders (rocprofv3 kernel trace over kbench's LZ4 rows).
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-lz4prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o k -- python3 tools/kbench.py --only ${ONLY:-lz4,lz4paths} --iters 3 > $OUT/kbench.jsonl 2>&1 || { tail -20 $OUT/kbench.jsonl; exit 1; }
cut -c1-120 $OUT/kbench.jsonl
