# round-6 call d: folded control collectives + start-up fetch rule; 2/4/8-rank rehearsals; single-command pull
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
bash tools/gpu/check.sh r6d swarm && \
RANKS=2 bash tools/gpu/check.sh r6d_n2 rehearsal > /dev/null && show r6d_n2 && \
RANKS=4 bash tools/gpu/check.sh r6d_n4 rehearsal > /dev/null && show r6d_n4 && \
RANKS=8 bash tools/gpu/check.sh r6d_n8 rehearsal > /dev/null && show r6d_n8 && \
timeout -k 10 300 python -m zest_amd.testing --help > /dev/null 2>&1; echo "testing module rc $?"
