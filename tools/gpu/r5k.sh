# round-5 call k: striping after the per-term thread split (capped 1250 MB/s and uncapped, 4 GB),
# GPU CLI vs host CLI on BG4-LZ4 bf16 weights
set -o pipefail
mkdir -p gpurun_out/r5k
STRIPE_ARGS="--rate-mbps 1250" bash tools/gpu/check.sh r5k/capped stripe || exit 1
bash tools/gpu/check.sh r5k/uncapped stripe || exit 1
CLI_MODE=bf16 bash tools/gpu/check.sh r5k cli
