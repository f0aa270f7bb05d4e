#!/bin/bash
# LZ4 ring-size sweep: correctness (kernel tests) and throughput per ZG_LZ4_RING (KiB per wave).
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/lz4ring
for r in ${RINGS:-4 8}; do
  ZG_LZ4_RING=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lz4ring/tests$r.log 2>&1 || { tail -20 gpurun_out/lz4ring/tests$r.log; exit 1; }
  ZG_LZ4_RING=$r timeout -k 10 300 python tools/kbench.py --only lz4,lz4big,lz4paths --iters 3 > gpurun_out/lz4ring/kbench$r.log 2>&1 || exit $?
  echo "== ring $r KiB: $(tail -1 gpurun_out/lz4ring/tests$r.log)"
  grep -h "ingest_" gpurun_out/lz4ring/kbench$r.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print('  %-32s %7.1f GB/s'%(d['kernel'],d['gbps']))"
done
