#!/bin/bash
# Engine pipeline shape A/B on the headline bench (Llama-3.1-70B, 1 GPU): "lanes" (H2D on the compute
# lanes) vs "copy" (one copy stream + slot events), for random bytes and for BG4-LZ4 bf16 chunks.
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-pipeline_ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for run in ${RUNS:-bf16:copy bf16:lanes random:copy random:lanes}; do
  mode=${run%%:*}; p=${run##*:}
  {
    ZEST_PIPELINE=$p timeout -k 10 500 python bench.py --mode $mode --steps 5 --warmup 1 > $OUT/${mode}_$p.log 2>&1 \
        || { tail -5 $OUT/${mode}_$p.log; exit 1; }
    echo "$mode $p: $(tail -1 $OUT/${mode}_$p.log | grep -o '"value": [0-9.]*')"
  }
done
