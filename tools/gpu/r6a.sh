# round-6 call a: streamed swarm rounds -- swarm GPU tests, peer-mapped tests, 2- and 4-rank rehearsals
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','exchange','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error','swarm_pull_streamed')})"; }
bash tools/gpu/check.sh r6a swarm ipc && \
RANKS=2 bash tools/gpu/check.sh r6a_n2 rehearsal > /dev/null && show r6a_n2 && \
RANKS=4 bash tools/gpu/check.sh r6a_n4 rehearsal > /dev/null && show r6a_n4
