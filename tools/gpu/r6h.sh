# round-6 call h: VMM re-import probe (fd-number hypothesis); fixed race/refill tests; MIN_ROUNDS 4 vs 8
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
mkdir -p gpurun_out/r6h
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 python -u tools/vmm_leak_probe.py --gb 4 --iters 3 --modes map,map_fresh,map_rev > gpurun_out/r6h/vmm_probe.log 2>&1; echo "probe rc $?"; tail -1 gpurun_out/r6h/vmm_probe.log | cut -c1-900
timeout -k 10 300 $PYT tests/test_gpu_device.py -k "hash_table_ordered or refilled" > gpurun_out/r6h/race_fixed.log 2>&1; echo "fixed rc $?"; tail -1 gpurun_out/r6h/race_fixed.log
ZEST_SWARM_MIN_ROUNDS=4 RANKS=4 bash tools/gpu/check.sh r6h_n4_mr4 rehearsal > /dev/null && show r6h_n4_mr4
ZEST_SWARM_MIN_ROUNDS=4 RANKS=8 bash tools/gpu/check.sh r6h_n8_mr4 rehearsal > /dev/null && show r6h_n8_mr4
