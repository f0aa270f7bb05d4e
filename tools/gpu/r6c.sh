# round-6 call c: streamed public path knobs at 4 ranks (head taper, fetch run-ahead); HBM seeding with piecewise D2H
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
RANKS=4 bash tools/gpu/check.sh r6c_n4 rehearsal > /dev/null && show r6c_n4 && \
ZEST_STREAM_AHEAD=1 RANKS=4 bash tools/gpu/check.sh r6c_n4_ahead1 rehearsal > /dev/null && show r6c_n4_ahead1 && \
ZEST_SWARM_HEAD_TAPER=0.0625,0.125,0.25,0.5 RANKS=4 bash tools/gpu/check.sh r6c_n4_head rehearsal > /dev/null && show r6c_n4_head && \
ZEST_STREAM_AHEAD=1 ZEST_SWARM_HEAD_TAPER=0.0625,0.125,0.25,0.5 RANKS=4 bash tools/gpu/check.sh r6c_n4_both rehearsal > /dev/null && show r6c_n4_both && \
bash tools/gpu/check.sh r6c seed
