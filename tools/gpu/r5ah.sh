# round-5 call ah: host micro-bench rows on the box's EPYC (new host LZ4/BG4 decoder row); GPU CLI vs
# host pull of bf16 weights (16 GB) from a warm `zest serve` seeder after the host decoder speed-up and
# the device pull's runs-only H2D
set -o pipefail
mkdir -p gpurun_out/r5ah
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
bash tools/gpu/check.sh r5ah hostbench || exit 1
CLI_MODE=bf16 CLIPEER_MB=16000 CLIPEER_TAG=_16g bash tools/gpu/check.sh r5ah clipeer
