# round-5 call ar: final record at HEAD: driver-shaped bench (20/5) and a 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out/r5ar
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
STEPS=20 WARMUP=5 bash tools/gpu/check.sh r5ar bench || exit 1
RANKS=2 bash tools/gpu/check.sh r5ar rehearsal
