# round-6 call b: 4-rank rehearsal of the streamed public path with device timelines; slot variants
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
RANKS=4 bash tools/gpu/check.sh r6b_n4 rehearsal > /dev/null && show r6b_n4 && \
ZEST_SWARM_STAGING_MB=256 ZEST_SWARM_SLOTS=6 RANKS=4 bash tools/gpu/check.sh r6b_n4_s256 rehearsal > /dev/null && show r6b_n4_s256 && \
ZEST_SWARM_STAGING_MB=1024 ZEST_SWARM_SLOTS=3 RANKS=4 bash tools/gpu/check.sh r6b_n4_s1024 rehearsal > /dev/null && show r6b_n4_s1024
