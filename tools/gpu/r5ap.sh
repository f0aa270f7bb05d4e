# round-5 call ap: the public-path row lands in the engine's arena (adopt_arena): 4- and 8-rank
# one-GPU rehearsals, then the N=1 bench
set -o pipefail
mkdir -p gpurun_out/r5ap/n8
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
summ() { grep -h "device free GB\|swarm_pull\] failed\|swarm_pull random\]" $1 | head -3 | cut -c1-400
  grep '^{"metric' $1 | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print({k: e[k] for k in e if k in ('bf16_GBps','random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_arena_reused','swarm_pull_error','swarm_pull_warmup_s','swarm_pull_first_call_alloc')})"; }
RANKS=4 bash tools/gpu/check.sh r5ap rehearsal || exit 1
summ gpurun_out/r5ap/rehearsal.log
RANKS=8 bash tools/gpu/check.sh r5ap/n8 rehearsal || exit 1
summ gpurun_out/r5ap/n8/rehearsal.log
bash tools/gpu/check.sh r5ap bench
