# round-5 call ad: is the headline lower when bench.py runs both data modes (63.2 on two boxes) than
# bf16 alone (64.3 on four)?  Same box: default modes, then --modes bf16
set -o pipefail
mkdir -p gpurun_out/r5ad
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
bash tools/gpu/check.sh r5ad bench || exit 1
BENCH_MODES=bf16 bash tools/gpu/check.sh r5ad benchA
