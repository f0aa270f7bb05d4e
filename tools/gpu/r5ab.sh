# round-5 call ab: scan at 64 positions per thread; scan tests; gpubench with the scan; the 70B bf16
# engine bench with the serial walk (A) vs the parallel walk (B)
set -o pipefail
mkdir -p gpurun_out/r5ab/scan
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "index_scan or ingest_matches" > gpurun_out/r5ab/scan_tests.log 2>&1 || { tail -30 gpurun_out/r5ab/scan_tests.log; exit 1; }
tail -1 gpurun_out/r5ab/scan_tests.log
ZEST_INDEX_SCAN=1 bash tools/gpu/check.sh r5ab/scan gprof || exit 1
GPUBENCH_ENV="ZEST_INDEX_SCAN=1" bash tools/gpu/check.sh r5ab/scan gpubench || exit 1
BENCH_MODES=bf16 BENCH_ENV_A="ZEST_INDEX_SCAN=0" BENCH_ENV_B="ZEST_INDEX_SCAN=1" bash tools/gpu/check.sh r5ab benchA benchB
