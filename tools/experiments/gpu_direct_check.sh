#!/bin/bash
# Device-direct pull: GPU device tests (direct pull, repair, swarm_pull, CLI --gpus), then the
# Llama-3.1-8B loopback bench with a Chrome trace of the fetch pipeline.
export ZEST_SKIP_BUILD=1
OUT=gpurun_out/${OUT_TAG:-direct}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_device.py -v -m gpu -x --timeout 300 --timeout-method thread > $OUT/device_tests.log 2>&1
rc=$?; echo "device tests rc=$rc"; tail -2 $OUT/device_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/device_tests.log | head -30; exit $rc; fi
ZEST_TRACE=$PWD/$OUT/trace.json timeout -k 10 300 python tools/direct_bench.py --model llama-3.1-8b --skip-host --out $OUT/direct.json > $OUT/direct.log 2>&1 || { tail -20 $OUT/direct.log; exit 1; }
grep -v amdgpu.ids $OUT/direct.log | head -4
