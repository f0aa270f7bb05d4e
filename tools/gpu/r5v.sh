# round-5 call v: GPU-side exchange readiness (shared ready counters + hipStreamWaitValue32, no host
# barrier per round): unit test, the peer-mapped 2-rank tests, 2-rank rehearsal signals on/off;
# swarm GPU tests; the public path on the 70B bf16 world
set -o pipefail
mkdir -p gpurun_out/r5v
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_ipc.py \
  -k "signals_gate" > gpurun_out/r5v/signals_unit.log 2>&1 || { tail -30 gpurun_out/r5v/signals_unit.log; exit 1; }
grep -E "PASSED|SKIPPED" gpurun_out/r5v/signals_unit.log
bash tools/gpu/check.sh r5v ipc || exit 1
run() {  # tag, env...
  local tag=$1; shift
  env ZEST_BENCH_BACKEND=gloo "$@" timeout -k 10 400 python -u bench.py --gpus 2 --model llama-3.1-8b --modes bf16,random \
    --steps 3 --warmup 1 > gpurun_out/r5v/$tag.log 2>&1 || { echo "[r5v] $tag failed"; tail -30 gpurun_out/r5v/$tag.log; exit 1; }
  echo "== $tag $*"; grep -h "GB/s aggregate" gpurun_out/r5v/$tag.log | grep -v "bench r1"
  tail -1 gpurun_out/r5v/$tag.log | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; print({k: v for k, v in d['extra'].items() if 'wait' in k or 'ms_per' in k or 'signals' in k})"
}
run sig_on ZEST_IPC_SIGNALS=1
run sig_off ZEST_IPC_SIGNALS=0
bash tools/gpu/check.sh r5v swarm || exit 1
SR_MODEL=llama-3.1-70b SR_MODES=bf16 bash tools/gpu/check.sh r5v swarmrow
