# round-5 call r: HBM seeding (Mixtral-8x7B, responses/s + GB/s); striping after the host registry lookup
set -o pipefail
mkdir -p gpurun_out/r5r
bash tools/gpu/check.sh r5r seed || exit 1
STRIPE_ARGS="--rate-mbps 1250" bash tools/gpu/check.sh r5r/capped stripe || exit 1
bash tools/gpu/check.sh r5r/uncapped stripe
