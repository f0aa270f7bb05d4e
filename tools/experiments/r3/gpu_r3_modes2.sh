#!/bin/bash
# Round 3: second-mode slowdown diagnosis (same mode twice; bf16 then random) with arena + staging reuse.
OUT=gpurun_out/r3modes2; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --modes random,random > $OUT/rr.log 2>&1 || { tail -30 $OUT/rr.log; exit 1; }
grep -h "aggregate" $OUT/rr.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --modes bf16,random > $OUT/br.log 2>&1 || { tail -30 $OUT/br.log; exit 1; }
grep -h "aggregate" $OUT/br.log
