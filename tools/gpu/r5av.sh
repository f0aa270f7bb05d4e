# round-5 call av: 8 ranks on the one GPU, public-path row with 1 GiB vs 256 MiB staging slots
set -o pipefail
mkdir -p gpurun_out/r5av
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp ZEST_BENCH_BACKEND=gloo
run() { local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --gpus 8 --model llama-3.1-8b --modes random --steps 3 --warmup 1 \
    --swarm-steps 3 ${SW_ARGS:-} > gpurun_out/r5av/$tag.log 2>&1 || { echo "[r5av] $tag failed"; tail -20 gpurun_out/r5av/$tag.log; exit 1; }
  echo "== $tag $*"; grep -h "GB/s aggregate" gpurun_out/r5av/$tag.log | grep -v "bench r"
  grep '^{"metric' gpurun_out/r5av/$tag.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print(e.get('swarm_pull_step_s'), e.get('swarm_pull_phases',{}).get('fetch_s'), e.get('swarm_pull_phases',{}).get('agree_s'), e.get('swarm_pull_error'))"; }
run n8_256 ZEST_SWARM_STAGING_MB=256
run n8_1g ZEST_SWARM_STAGING_MB=1024
