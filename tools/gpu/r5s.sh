# round-5 call s (fresh container, rebuilt tree): full GPU suite, smoke and the default bench at HEAD;
# HBM seeding (responses/s + GB/s); striping capped/uncapped
set -o pipefail
mkdir -p gpurun_out/r5s
bash tools/gpu/check.sh r5s tests smoke bench || exit 1
bash tools/gpu/check.sh r5s seed || exit 1
STRIPE_ARGS="--rate-mbps 1250" bash tools/gpu/check.sh r5s/capped stripe || exit 1
bash tools/gpu/check.sh r5s/uncapped stripe
