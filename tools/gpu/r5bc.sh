# round-5 call bc: 4 ranks on the one GPU with the half-round default, 5 timed public-path pulls
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp ZEST_BENCH_BACKEND=gloo
mkdir -p gpurun_out/r5bc
timeout -k 10 400 python -u bench.py --gpus 4 --model llama-3.1-8b --modes random --steps 3 --warmup 1 \
  --swarm-steps 5 > gpurun_out/r5bc/n4_512_s5.log 2>&1 || { tail -20 gpurun_out/r5bc/n4_512_s5.log; exit 1; }
grep -h "GB/s aggregate" gpurun_out/r5bc/n4_512_s5.log | grep -v "bench r"
grep '^{"metric' gpurun_out/r5bc/n4_512_s5.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print(e.get('swarm_pull_step_s'), e.get('swarm_pull_error'))"
