# round-5 call i: Merkle numerics after the LDS-stride change, counter table, striping at Llama-8B size
set -o pipefail
mkdir -p gpurun_out/r5i
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "merkle or ingest_matches or device_puller_pipelines" > gpurun_out/r5i/kernels.log 2>&1 || { tail -30 gpurun_out/r5i/kernels.log; exit 1; }
tail -1 gpurun_out/r5i/kernels.log
bash tools/gpu/check.sh r5i pmctable || exit 1
STRIPE_MB=16000 STRIPE_ARGS="--rate-mbps 1250" bash tools/gpu/check.sh r5i/capped16g stripe
