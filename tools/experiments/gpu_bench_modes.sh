#!/bin/bash
# 1-GPU headline bench in both data modes (random bytes = headline; bf16 = BG4-LZ4 chunks decoded on the GPU).
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-benchmodes}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --mode bf16 > $OUT/bench_n1_bf16.log 2>&1 || exit $?
tail -1 $OUT/bench_n1_bf16.log | cut -c1-200
if [ -n "$RING_AB" ]; then
  ZG_LZ4_SEQ=0 timeout -k 10 600 python bench.py --steps 3 --warmup 1 --mode bf16 > $OUT/bench_n1_bf16_ring.log 2>&1 || exit $?
  tail -1 $OUT/bench_n1_bf16_ring.log | cut -c1-200
fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $OUT/bench_n1.log 2>&1 || exit $?
tail -1 $OUT/bench_n1.log | cut -c1-200
