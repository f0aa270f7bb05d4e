# round-5 call q: GPU CLI vs host at Llama-3.1-8B size (16 GB) from a warm `zest serve` seeder
set -o pipefail
mkdir -p gpurun_out/r5q
CLI_MODE=bf16 CLIPEER_MB=16000 CLIPEER_TAG=_16g bash tools/gpu/check.sh r5q clipeer || exit 1
CLI_MODE=random CLIPEER_MB=16000 CLIPEER_TAG=_16g bash tools/gpu/check.sh r5q clipeer
