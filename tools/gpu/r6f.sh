# round-6 call f: VMM release probe; refill test; 4/8-rank rehearsals with adaptive streamed rounds;
# 4 ranks with 16 HW queues per process (head-of-line blocking hypothesis)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
mkdir -p gpurun_out/r6f
timeout -k 10 400 python -u tools/vmm_leak_probe.py --gb 8 --iters 3 > gpurun_out/r6f/vmm_probe.log 2>&1; echo "probe rc $?"; tail -1 gpurun_out/r6f/vmm_probe.log | cut -c1-600
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_device.py -k "refilled or write_behind" > gpurun_out/r6f/refill.log 2>&1; echo "refill rc $?"; tail -2 gpurun_out/r6f/refill.log
RANKS=4 bash tools/gpu/check.sh r6f_n4 rehearsal > /dev/null && show r6f_n4 && \
RANKS=8 bash tools/gpu/check.sh r6f_n8 rehearsal > /dev/null && show r6f_n8 && \
ZEST_BENCH_HW_QUEUES=16 RANKS=4 bash tools/gpu/check.sh r6f_n4_hwq16 rehearsal > /dev/null && show r6f_n4_hwq16
