# round-5 call am: 8-rank rehearsal on the one GPU (the driver's N=8 code paths: 7 peers per rank,
# GPU-side readiness, K8 over 7 segments, VMM mapping turns for 8 ranks, public-path row with reuse_arena)
set -o pipefail
mkdir -p gpurun_out/r5am
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
RANKS=8 bash tools/gpu/check.sh r5am rehearsal || exit 1
grep '^{"metric' gpurun_out/r5am/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print({k: e[k] for k in e if k in ('bf16_GBps','random_GBps','ipc_signals','ipc_host_wait_ms_per_step','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_arena_reused','swarm_pull_exchange','swarm_pull_error')}); print(d['config']['phase_s'], d['config']['exchange'], d['config']['exchange_autotune_s'])"
