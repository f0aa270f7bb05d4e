# round-5 call z: per-kernel times of gpubench 256 MiB with the parallel header walk (ZEST_INDEX_SCAN=1)
set -o pipefail
mkdir -p gpurun_out/r5z
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp ZEST_INDEX_SCAN=1
bash tools/gpu/check.sh r5z gprof
