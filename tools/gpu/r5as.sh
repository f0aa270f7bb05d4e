# round-5 call as: public-path row at N=2/4 (one GPU) with 1 GiB staging slots (default: one batch per
# 1 GiB round, no pipelining inside a round) vs 256 MiB slots (4 batches per round)
set -o pipefail
mkdir -p gpurun_out/r5as
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp ZEST_BENCH_BACKEND=gloo
run() { local tag=$1 n=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --gpus $n --model llama-3.1-8b --modes random --steps 3 --warmup 1 \
    > gpurun_out/r5as/$tag.log 2>&1 || { echo "[r5as] $tag failed"; tail -20 gpurun_out/r5as/$tag.log; exit 1; }
  echo "== $tag $*"; grep -h "GB/s aggregate" gpurun_out/r5as/$tag.log | grep -v "bench r"
  grep '^{"metric' gpurun_out/r5as/$tag.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print(e.get('swarm_pull_step_s'), e.get('swarm_pull_phases',{}).get('fetch_s'), e.get('swarm_pull_error'))"; }
run n2_1g 2 ZEST_SWARM_STAGING_MB=1024
run n2_256 2 ZEST_SWARM_STAGING_MB=256
run n4_1g 4 ZEST_SWARM_STAGING_MB=1024
run n4_256 4 ZEST_SWARM_STAGING_MB=256
