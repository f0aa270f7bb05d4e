# round-6 call o: exchange-window shape in the 4/8-rank rehearsals (random mode, 4 timed public pulls);
# quarter-round staging slots at 4 and 8 ranks (no step > 1.5x the median: VERDICT r5 item 2)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; s=sorted(e.get('swarm_pull_step_s',[0])); print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k == 'swarm_pull_step_s'}, 'max/median %.2f' % (s[-1]/s[len(s)//2]))"; }
export REHEARSAL_ARGS="--modes random --swarm-steps 4"
run() { tag=$1; shift; env "$@" bash tools/gpu/check.sh $tag rehearsal > /dev/null && show $tag; }
run r6o_n4_w256x4 RANKS=4 && \
run r6o_n4_w512x4 RANKS=4 ZEST_SWARM_WINDOW_MB=512 && \
run r6o_n4_w256x8 RANKS=4 ZEST_SWARM_WINDOW_SLOTS=8 && \
run r6o_n8_w256x4 RANKS=8 && \
run r6o_n8_w512x4 RANKS=8 ZEST_SWARM_WINDOW_MB=512 && \
run r6o_n8_w256x8 RANKS=8 ZEST_SWARM_WINDOW_SLOTS=8 && \
REHEARSAL_ARGS="--modes random --swarm-steps 5" run r6o_n4_quarter RANKS=4 ZEST_SWARM_STAGING_MB=256 && \
REHEARSAL_ARGS="--modes random --swarm-steps 5" run r6o_n8_quarter RANKS=8 ZEST_SWARM_STAGING_MB=256
