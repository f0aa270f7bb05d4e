#!/bin/bash
# Round-2 check: GPU tests, smoke, 1-GPU headline bench, 2-rank gloo rehearsal of the multi-rank bench.
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-r2c}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $OUT/bench_n1.log 2>&1 || exit $?
tail -1 $OUT/bench_n1.log | cut -c1-220
if [ -n "$REHEARSE" ]; then
  export ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 ZEST_BENCH_WATCHDOG=150
  timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29561 bench.py --gpus 2 --model llama-3.1-8b --exchange auto --steps 2 --warmup 1 \
      > $OUT/rehearsal_n2.log 2>&1 || { grep -v amdgpu.ids $OUT/rehearsal_n2.log | tail -40; exit 1; }
  tail -1 $OUT/rehearsal_n2.log | cut -c1-300
fi
