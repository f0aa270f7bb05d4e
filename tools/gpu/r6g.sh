# round-6 call g: the hash-table race (round 5's stall): negative control (race restored) must fail,
# the fix must pass; 4 ranks with 16 HW queues again; VMM release probe; refill test
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
mkdir -p gpurun_out/r6g
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
ZEST_SWARM_UNORDERED_TABLES=1 timeout -k 10 300 $PYT tests/test_gpu_device.py -k hash_table_ordered > gpurun_out/r6g/race_restored.log 2>&1; echo "race restored rc $? (expect 1)"; grep -E "passed|failed" gpurun_out/r6g/race_restored.log | tail -1
timeout -k 10 300 $PYT tests/test_gpu_device.py -k "hash_table_ordered or refilled" > gpurun_out/r6g/race_fixed.log 2>&1; echo "fixed rc $?"; tail -1 gpurun_out/r6g/race_fixed.log
ZEST_BENCH_HW_QUEUES=16 RANKS=4 bash tools/gpu/check.sh r6g_n4_hwq16 rehearsal > /dev/null && show r6g_n4_hwq16
RANKS=4 bash tools/gpu/check.sh r6g_n4 rehearsal > /dev/null && show r6g_n4
timeout -k 10 400 python -u tools/vmm_leak_probe.py --gb 8 --iters 3 --modes map,map_rev > gpurun_out/r6g/vmm_probe.log 2>&1; echo "probe rc $?"; tail -1 gpurun_out/r6g/vmm_probe.log | cut -c1-600
