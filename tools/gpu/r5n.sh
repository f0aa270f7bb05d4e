# round-5 call n: GPU CLI vs host CLI from warm `zest serve` seeders (8 GB, bf16 and random)
set -o pipefail
mkdir -p gpurun_out/r5n
CLI_MODE=bf16 bash tools/gpu/check.sh r5n clipeer || exit 1
CLI_MODE=random bash tools/gpu/check.sh r5n clipeer
