# round-5 call aa: K4 link picks the chain out of candidates with look-alikes (no more all-terms fallback):
# scan tests, per-kernel times with ZEST_INDEX_SCAN=1, gpubench serial vs scan
set -o pipefail
mkdir -p gpurun_out/r5aa/scan
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "index_scan or ingest_matches" > gpurun_out/r5aa/scan_tests.log 2>&1 || { tail -30 gpurun_out/r5aa/scan_tests.log; exit 1; }
tail -1 gpurun_out/r5aa/scan_tests.log
ZEST_INDEX_SCAN=1 bash tools/gpu/check.sh r5aa/scan gprof || exit 1
bash tools/gpu/check.sh r5aa gpubench || exit 1
GPUBENCH_ENV="ZEST_INDEX_SCAN=1" bash tools/gpu/check.sh r5aa/scan gpubench
