# round-5 call r: HBM seeding (Mixtral-8x7B, responses/s + GB/s); striping after the host registry
# lookup; the public path on the 70B bf16 world (BG4-LZ4 decode inside swarm_pull)
set -o pipefail
mkdir -p gpurun_out/r5r
bash tools/gpu/check.sh r5r seed || exit 1
STRIPE_ARGS="--rate-mbps 1250" bash tools/gpu/check.sh r5r/capped stripe || exit 1
bash tools/gpu/check.sh r5r/uncapped stripe || exit 1
SR_MODEL=llama-3.1-70b SR_MODES=bf16 bash tools/gpu/check.sh r5r swarmrow
