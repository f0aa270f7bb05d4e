# round-6 call j: exchange windows (public path) -- swarm GPU tests incl. freed arenas; ipc tests; 2/4/8-rank rehearsals
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error','swarm_pull_exchange')})"; }
mkdir -p gpurun_out/r6j
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $PYT -v tests/test_gpu_device.py -k "swarm or refilled" > gpurun_out/r6j/swarm.log 2>&1 && grep -cE "PASSED" gpurun_out/r6j/swarm.log && tail -1 gpurun_out/r6j/swarm.log && \
RANKS=2 bash tools/gpu/check.sh r6j_n2 rehearsal > /dev/null && show r6j_n2 && \
RANKS=4 bash tools/gpu/check.sh r6j_n4 rehearsal > /dev/null && show r6j_n4 && \
RANKS=8 bash tools/gpu/check.sh r6j_n8 rehearsal > /dev/null && show r6j_n8
