# round-6 call z: the busiest threads of each rank (CPU seconds + voluntary / involuntary context
# switches) over the public-path row's timed calls, 8-rank rehearsal, random data
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
ZEST_BENCH_SPIN_PROBE=1 REHEARSAL_ARGS="--modes random --swarm-steps 3" RANKS=8 bash tools/gpu/check.sh r6z_n8 rehearsal > /dev/null && \
grep '^{"metric' gpurun_out/r6z_n8/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('row', e['swarm_pull_GBps'], 'engine', e['random_GBps'], e['swarm_pull_step_s'])
for r, t in enumerate(e['swarm_pull_busiest_threads'][:4]): print('rank', r, t)"
