# round-6 call aa: the ROCm runtime's polling completion thread in the 8-rank rehearsal: default
# dispatch vs AMD_DIRECT_DISPATCH=0 (busiest threads, row vs engine)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('$1 row', e['swarm_pull_GBps'], 'engine', e['random_GBps'], round(e['swarm_pull_GBps']/e['random_GBps'],3), e['swarm_pull_step_s'], 'engine rank0', d['config']['phase_s'].get('timed_thread_cpu_s'))
for r, t in enumerate(e['swarm_pull_busiest_threads'][:2]): print('   rank', r, t[:3])"; }
REHEARSAL_ARGS="--modes random --swarm-steps 3" RANKS=8 AMD_DIRECT_DISPATCH=0 bash tools/gpu/check.sh r6aa_dd0 rehearsal > /dev/null && show r6aa_dd0
