#!/bin/bash
# Round 3: fused place+hash kernel (numerics vs host oracle, kbench A/B), headline bench, native GPU
# CLI worker tests + host pull vs `zest pull --gpus 1`, full GPU suite.
OUT=gpurun_out/r3f; mkdir -p $OUT
export ZEST_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "ingest" -x -q --timeout 120 --timeout-method thread > $OUT/kern_tests.log 2>&1 || { tail -40 $OUT/kern_tests.log; exit 1; }
tail -1 $OUT/kern_tests.log
timeout -k 10 300 python -u tools/kbench.py --only fuse --iters 5 > $OUT/kbench_fuse.jsonl 2>&1 || { tail -20 $OUT/kbench_fuse.jsonl; exit 1; }
cat $OUT/kbench_fuse.jsonl | grep kernel
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep -h "aggregate" $OUT/bench.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_device.py -k "cli_pull_gpus" -x -q --timeout 200 --timeout-method thread > $OUT/cli_tests.log 2>&1 || { tail -40 $OUT/cli_tests.log; exit 1; }
tail -1 $OUT/cli_tests.log
timeout -k 10 600 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --out $OUT/cli_vs_host_8b.json > $OUT/cli_vs_host.log 2>&1 || { tail -30 $OUT/cli_vs_host.log; exit 1; }
grep -h "^\[" $OUT/cli_vs_host.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
