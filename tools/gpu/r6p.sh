# round-6 call p: CPU seconds per public-path call vs the engine's timed loop (4/8 ranks, one GPU);
# agreements on their own thread (default) vs on the pulling thread; first staging batch 32 MiB;
# bf16-only row at 8 ranks
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)  nproc: $(nproc)"
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; ph=d['config']['phase_s']
sp=e.get('swarm_pull_step_phases') or []
cpu=[round(sum(st[i]['cpu_s'] for st in sp),2) for i in range(len(sp[0]))] if sp else None
print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k == 'swarm_pull_step_s'}, 'engine timed_s', ph.get('timed_s'), 'engine cpu_s(rank0)', ph.get('timed_cpu_s'), 'row cpu_s per call (all ranks)', cpu)"; }
run() { tag=$1; shift; env "$@" bash tools/gpu/check.sh $tag rehearsal > /dev/null && show $tag; }
export REHEARSAL_ARGS="--modes random --swarm-steps 3"
mkdir -p gpurun_out/r6p
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -v tests/test_gpu_device.py -k "swarm" > gpurun_out/r6p/swarm.log 2>&1; rc=$?; echo "swarm tests rc $rc: $(tail -1 gpurun_out/r6p/swarm.log)"; [ $rc = 0 ] && \
run r6p_n4 RANKS=4 && \
run r6p_n4_nothread RANKS=4 ZEST_SWARM_AGREE_THREAD=0 && \
run r6p_n8 RANKS=8 && \
run r6p_n8_nothread RANKS=8 ZEST_SWARM_AGREE_THREAD=0 && \
run r6p_n8_fb32 RANKS=8 ZEST_FIRST_BATCH_MB=32 && \
REHEARSAL_ARGS="--modes bf16 --swarm-steps 3" run r6p_n8_bf16 RANKS=8
