# round-6 call s: host waits that sleep instead of polling (native event waits, swarm_pull's
# verify / settle waits): swarm GPU tests, N = 1 bench (both rows), 4/8-rank rehearsals
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/$2.log | tail -1 | python -c "
import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']
sp=e.get('swarm_pull_step_phases') or []
cpu=[round(sum(st[i]['cpu_s'] for st in sp),2) for i in range(len(sp[0]))] if sp else None
print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k == 'swarm_pull_step_s'}, 'row cpu_s/call', cpu)
for r, t in enumerate((e.get('swarm_pull_thread_cpu_s') or [])[:2]): print('   row rank', r, t)"; }
mkdir -p gpurun_out/r6s
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -v tests/test_gpu_device.py -k "swarm" > gpurun_out/r6s/swarm.log 2>&1; rc=$?; echo "swarm tests rc $rc: $(tail -1 gpurun_out/r6s/swarm.log)"; [ $rc = 0 ] && \
bash tools/gpu/check.sh r6s bench > /dev/null && show r6s bench && \
REHEARSAL_ARGS="--swarm-steps 3" RANKS=4 bash tools/gpu/check.sh r6s_n4 rehearsal > /dev/null && show r6s_n4 rehearsal && \
REHEARSAL_ARGS="--swarm-steps 3" RANKS=8 bash tools/gpu/check.sh r6s_n8 rehearsal > /dev/null && show r6s_n8 rehearsal
