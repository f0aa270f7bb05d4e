#!/bin/bash
# Two-phase LZ4 decoder: GPU kernel tests, then kbench LZ4 rows for the new decoder and the
# LDS-ring decoder (ZG_LZ4_SEQ=0).
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-lz4seq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -m gpu -x --timeout 120 --timeout-method thread > $OUT/kernel_tests.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 $OUT/kernel_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/kernel_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python tools/kbench.py --only lz4,lz4big,lz4paths --iters 5 > $OUT/kbench_seq.jsonl 2>&1 || { tail -20 $OUT/kbench_seq.jsonl; exit 1; }
cut -c1-160 $OUT/kbench_seq.jsonl
ZG_LZ4_SEQ=0 timeout -k 10 300 python tools/kbench.py --only lz4,lz4big,lz4paths --iters 5 > $OUT/kbench_ring.jsonl 2>&1 || exit 1
cut -c1-160 $OUT/kbench_ring.jsonl
