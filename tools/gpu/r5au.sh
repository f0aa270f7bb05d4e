# round-5 call au: final 8-rank one-GPU rehearsal at HEAD (quarter-round staging, adopted arena,
# automatic arena reuse, GPU-side readiness)
set -o pipefail
mkdir -p gpurun_out/r5au
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
RANKS=8 bash tools/gpu/check.sh r5au rehearsal || exit 1
grep -h "split check\|swarm_pull\] failed\|swarm_pull random\]" gpurun_out/r5au/rehearsal.log | head -3 | cut -c1-400
grep '^{"metric' gpurun_out/r5au/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print({k: e[k] for k in e if k in ('bf16_GBps','random_GBps','ipc_signals','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_arena_reused','swarm_pull_error')})"
