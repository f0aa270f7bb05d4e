# round-6 call y: Python profile of the public-path row's timed calls (pulling thread + agreement
# thread) in the 8-rank rehearsal, random data
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6y
ZEST_BENCH_PYPROF=1 ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 timeout -k 10 600 python -u bench.py --gpus 8 --model llama-3.1-8b \
  --steps 3 --warmup 1 --modes random --swarm-steps 3 > gpurun_out/r6y/rehearsal.log 2>&1 || { echo "rehearsal failed rc $?"; tail -20 gpurun_out/r6y/rehearsal.log; exit 1; }
grep '^{"metric' gpurun_out/r6y/rehearsal.log | tail -1 | cut -c1-400
grep -n -A30 "^\[bench\] \[swarm_pull\] Python profile" gpurun_out/r6y/rehearsal.log | head -40
