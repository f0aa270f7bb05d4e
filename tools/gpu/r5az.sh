# round-5 call az: half-round staging default above 4 ranks: swarm GPU tests + 8-rank rehearsal
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
RANKS=8 bash tools/gpu/check.sh r5az swarm rehearsal || exit 1
grep '^{"metric' gpurun_out/r5az/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print(d['value'], {k: e[k] for k in e if k in ('bf16_GBps','random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_arena_reused','swarm_pull_error')})"
