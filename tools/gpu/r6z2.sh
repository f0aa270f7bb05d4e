# round-6 call z2: the ROCr thread that polls (~1 CPU-s per 3 public pulls per rank): device timing
# events on (bench default) vs off in the 8-rank rehearsal, random data
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('$1 row', e['swarm_pull_GBps'], 'engine', e['random_GBps'], round(e['swarm_pull_GBps']/e['random_GBps'],3), e['swarm_pull_step_s'])
for r, t in enumerate(e['swarm_pull_busiest_threads'][:2]): print('   rank', r, t[:3])"; }
REHEARSAL_ARGS="--modes random --swarm-steps 3" RANKS=8 bash tools/gpu/check.sh r6z2_timing rehearsal > /dev/null && show r6z2_timing && \
ZEST_DEVICE_TIMING=0 REHEARSAL_ARGS="--modes random --swarm-steps 3" RANKS=8 bash tools/gpu/check.sh r6z2_notiming rehearsal > /dev/null && show r6z2_notiming
