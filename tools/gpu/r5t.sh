# round-5 call t: 2-rank rehearsal (ranks share the GPU, gloo control, peer-mapped arenas), Llama-3.1-8B:
# why bf16 ran 750 ms/step in r5j against 289 in round 4 -- ipc lag 1 vs 2, copy vs lanes pipeline
set -o pipefail
mkdir -p gpurun_out/r5t
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp ZEST_BENCH_BACKEND=gloo
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --gpus 2 --model llama-3.1-8b --modes bf16,random --steps 3 --warmup 1 \
    > gpurun_out/r5t/$tag.log 2>&1 || { echo "[r5t] $tag failed"; tail -30 gpurun_out/r5t/$tag.log; exit 1; }
  echo "== $tag $*"; grep -h "GB/s aggregate" gpurun_out/r5t/$tag.log | grep -v "bench r1"
  tail -1 gpurun_out/r5t/$tag.log | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; print({k: v for k, v in d['extra'].items() if 'wait' in k or 'ms_per' in k})"
}
run lag1 ZEST_IPC_LAG=1
run lag2 ZEST_IPC_LAG=2
run lag2_lanes ZEST_IPC_LAG=2 ZEST_PIPELINE=lanes
run lag2_nofuse ZEST_IPC_LAG=2 ZG_FUSED_HASH=0
