# round-6 call ii: closing (after the decoder spill fix) 2/4/8-rank rehearsals at the final code (both data modes, 3 timed public
# pulls each): row / engine per mode, the agreement's own cost, the busiest thread per rank
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('$1', {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k in ('swarm_pull_step_s','swarm_pull_agree_own_frac')})"; }
for n in 2 4 8; do
  REHEARSAL_ARGS="--swarm-steps 3" RANKS=$n bash tools/gpu/check.sh r6mm_n$n rehearsal > /dev/null && show r6mm_n$n || exit 1
done
