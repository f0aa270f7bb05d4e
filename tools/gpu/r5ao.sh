# round-5 call ao: does releasing the engine's peer-mapped arenas free device memory before the
# public-path row? (4 ranks sharing the GPU; free memory before/after release and after the barrier)
set -o pipefail
mkdir -p gpurun_out/r5ao
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
RANKS=4 bash tools/gpu/check.sh r5ao rehearsal || exit 1
grep -h "device free GB\|swarm_pull\] failed" gpurun_out/r5ao/rehearsal.log | head -8 | cut -c1-300
