# round-6 call dd: kernel + copy trace of every rank in the 8-rank bf16 rehearsal; GPU activity inside
# the public-path row's timed window (ZEST_BENCH_MARK=1 sleep kernels bracket it).
# NOTE: every rank died with SIGSEGV at start-up under --kernel-trace --memory-copy-trace (host side;
# the 1-rank `check.sh prof` kernel trace works): not rerun -- see profiles/r6/stream_priority_r6cc/.
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6dd
ZEST_BENCH_MARK=1 ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 timeout -k 10 700 rocprofv3 --kernel-trace --memory-copy-trace \
  -d gpurun_out/r6dd/trace -o t --output-format csv -- python3 bench.py --gpus 8 --model llama-3.1-8b --steps 3 --warmup 1 \
  --modes bf16 --swarm-steps 3 > gpurun_out/r6dd/rehearsal.log 2>&1 || { echo "traced rehearsal failed rc $?"; tail -5 gpurun_out/r6dd/rehearsal.log; exit 1; }
grep '^{"metric' gpurun_out/r6dd/rehearsal.log | tail -1 | cut -c1-300
python tools/gpu/row_window.py gpurun_out/r6dd/trace | tee gpurun_out/r6dd/row_window.md
du -sh gpurun_out/r6dd/trace
find gpurun_out/r6dd/trace -name "*.csv" -size +20M -delete
