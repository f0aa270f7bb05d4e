# round-5 call y: the K4 parallel header walk after the LZ4-magic test on compressed candidates
# (6e580ce): scan tests, gpubench 256 MiB with the serial walk (default) and with ZEST_INDEX_SCAN=1
set -o pipefail
mkdir -p gpurun_out/r5y/scan
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "index_scan or ingest_matches" > gpurun_out/r5y/scan_tests.log 2>&1 || { tail -30 gpurun_out/r5y/scan_tests.log; exit 1; }
tail -1 gpurun_out/r5y/scan_tests.log
bash tools/gpu/check.sh r5y gpubench || exit 1
GPUBENCH_ENV="ZEST_INDEX_SCAN=1" bash tools/gpu/check.sh r5y/scan gpubench
