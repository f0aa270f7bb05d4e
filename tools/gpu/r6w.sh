# round-6 call w: the full GPU test suite, smoke, the N = 1 bench and the 8-rank rehearsal (both modes)
# at the dynamic-schedule decoder
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/$2.log | tail -1 | python -c "
import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']
print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k in ('swarm_pull_step_s', 'swarm_pull_agree_own_frac')})"; }
bash tools/gpu/check.sh r6w tests smoke && \
bash tools/gpu/check.sh r6w bench > /dev/null && show r6w bench && \
REHEARSAL_ARGS="--swarm-steps 3" RANKS=8 bash tools/gpu/check.sh r6w_n8 rehearsal > /dev/null && show r6w_n8 rehearsal
