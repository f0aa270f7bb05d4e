# round-5 call al: swarm_pull reuse_arena on the GPU: swarm GPU tests; 4-rank rehearsal (public-path
# row timed pulls land in the warm-up pull's VMM arena + mappings); N=1 bench
set -o pipefail
mkdir -p gpurun_out/r5al
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
bash tools/gpu/check.sh r5al swarm || exit 1
RANKS=4 bash tools/gpu/check.sh r5al rehearsal || exit 1
tail -1 gpurun_out/r5al/rehearsal.log | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print({k: e[k] for k in e if k in ('bf16_GBps','random_GBps','ipc_signals','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_arena_reused','swarm_pull_phases')})"
bash tools/gpu/check.sh r5al bench
