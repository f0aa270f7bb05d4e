# round-6 call e: swarm GPU tests; 2/4/8-rank rehearsals (folded collectives, start-up fetch rule);
# single-command replicated pull (2 ranks); VMM release probe
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error')})"; }
mkdir -p gpurun_out/r6e
bash tools/gpu/check.sh r6e swarm && \
RANKS=2 bash tools/gpu/check.sh r6e_n2 rehearsal > /dev/null && show r6e_n2 && \
RANKS=4 bash tools/gpu/check.sh r6e_n4 rehearsal > /dev/null && show r6e_n4 && \
RANKS=8 bash tools/gpu/check.sh r6e_n8 rehearsal > /dev/null && show r6e_n8 && \
timeout -k 10 300 python -u tools/replicate_rehearsal.py --ranks 2 --model gpt2 > gpurun_out/r6e/replicate.log 2>&1 && tail -1 gpurun_out/r6e/replicate.log | cut -c1-700 && \
timeout -k 10 300 python -u tools/experiments/vmm_leak_probe.py --gb 8 --iters 3 > gpurun_out/r6e/vmm_probe.log 2>&1 && tail -1 gpurun_out/r6e/vmm_probe.log
