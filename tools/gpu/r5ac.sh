# round-5 call ac: checkpoint after the GPU-side exchange readiness, runs-only H2D and the parallel
# header walk default: full GPU suite, smoke, default bench (N=1), 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out/r5ac
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
bash tools/gpu/check.sh r5ac tests smoke bench || exit 1
RANKS=2 bash tools/gpu/check.sh r5ac rehearsal
