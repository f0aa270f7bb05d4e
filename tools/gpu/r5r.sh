# round-5 call r: HBM seeding (Mixtral-8x7B, responses/s + GB/s); striping after the host registry
# lookup; the public path on the 70B bf16 world (BG4-LZ4 decode inside swarm_pull)
set -o pipefail
mkdir -p gpurun_out/r5r
bash tools/gpu/check.sh r5r seed || exit 1
STRIPE_ARGS="--rate-mbps 1250" bash tools/gpu/check.sh r5r/capped stripe || exit 1
bash tools/gpu/check.sh r5r/uncapped stripe || exit 1
SR_MODEL=llama-3.1-70b SR_MODES=bf16 bash tools/gpu/check.sh r5r swarmrow || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "index_scan or ingest_matches" > gpurun_out/r5r/scan_tests.log 2>&1 && tail -1 gpurun_out/r5r/scan_tests.log &&
mkdir -p gpurun_out/r5r/scan && GPUBENCH_ENV="ZEST_INDEX_SCAN=1" bash tools/gpu/check.sh r5r/scan gpubench
