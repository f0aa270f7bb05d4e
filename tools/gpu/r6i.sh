# round-6 call i: one-way VMM import probe; refill test; H2D merge-gap and slots knobs at 4 ranks
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
mkdir -p gpurun_out/r6i
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 python -u tools/vmm_oneway_probe.py --gb 4 > gpurun_out/r6i/oneway.log 2>&1; echo "oneway rc $?"; tail -1 gpurun_out/r6i/oneway.log | cut -c1-900
timeout -k 10 300 $PYT tests/test_gpu_device.py -k "refilled" > gpurun_out/r6i/refill.log 2>&1; echo "refill rc $?"; tail -1 gpurun_out/r6i/refill.log
ZEST_H2D_MERGE_GAP=16777216 RANKS=4 bash tools/gpu/check.sh r6i_n4_merge rehearsal > /dev/null && show r6i_n4_merge
ZEST_SWARM_SLOTS=3 RANKS=4 bash tools/gpu/check.sh r6i_n4_slots3 rehearsal > /dev/null && show r6i_n4_slots3
ZEST_SWARM_SLOTS=6 RANKS=4 bash tools/gpu/check.sh r6i_n4_slots6 rehearsal > /dev/null && show r6i_n4_slots6
