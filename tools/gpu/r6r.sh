# round-6 call r: where each rank's CPU goes in the 8-rank rehearsal (per-thread CPU seconds over the
# timed public pulls and the engine's timed steps); events waited with blocking sync vs polling
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; ph=d['config']['phase_s']
sp=e.get('swarm_pull_step_phases') or []
cpu=[round(sum(st[i]['cpu_s'] for st in sp),2) for i in range(len(sp[0]))] if sp else None
print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k == 'swarm_pull_step_s'}, 'row cpu_s/call', cpu)
print('   engine rank0 threads', ph.get('timed_thread_cpu_s'))
for r, t in enumerate(e.get('swarm_pull_thread_cpu_s') or []): print('   row rank', r, t)"; }
run() { tag=$1; shift; env "$@" bash tools/gpu/check.sh $tag rehearsal > /dev/null && show $tag; }
export REHEARSAL_ARGS="--modes random --swarm-steps 3"
run r6r_n8 RANKS=8 && \
run r6r_n8_block RANKS=8 ZEST_EVENT_BLOCKING=1
