# round-5 call w: why the public path's bf16 H2D copies run at 49.8 GB/s (engine: 56.3): per-copy
# rates of engine vs public-path copies by overlap with decode/hash kernels (70B bf16, kernel +
# memory-copy trace only)
set -o pipefail
mkdir -p gpurun_out/r5w
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
ZEST_BENCH_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r5w/ct -o ct -- \
  python3 bench.py --model llama-3.1-70b --modes bf16 --steps 2 --warmup 1 --swarm-steps 2 --swarm-warmup 0 \
  > gpurun_out/r5w/ct.log 2>&1 || { tail -30 gpurun_out/r5w/ct.log; exit 1; }
grep -h "aggregate" gpurun_out/r5w/ct.log
python tools/gpu/copy_rates.py gpurun_out/r5w/ct > gpurun_out/r5w/copy_rates.txt 2>&1; cat gpurun_out/r5w/copy_rates.txt
python tools/gpu/overlap.py gpurun_out/r5w/ct --between spin_kernel > gpurun_out/r5w/overlap_swarm.txt 2>&1; cat gpurun_out/r5w/overlap_swarm.txt
rm -rf gpurun_out/r5w/ct
