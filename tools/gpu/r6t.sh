# round-6 call t: bf16 public-path row vs rounds per share (ZEST_SWARM_MIN_ROUNDS 8 / 4 / 2): the GPU
# LZ4 decode of a 256 MiB batch runs at ~85 GB/s against ~136 at 1 GiB (one wave of blocks)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']
sp=e.get('swarm_pull_step_phases') or []
kb=[round(sum(st[i]['timeline'].get('kernel_busy_ms',0) for st in sp)/len(sp),1) for i in range(len(sp[0]))] if sp else None
print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k == 'swarm_pull_step_s'}, 'mean kernel_busy_ms/rank', kb)"; }
run() { tag=$1; shift; env "$@" bash tools/gpu/check.sh $tag rehearsal > /dev/null && show $tag; }
export REHEARSAL_ARGS="--modes bf16 --swarm-steps 3 --swarm-warmup 2"
run r6t_n8_r8 RANKS=8 && \
run r6t_n8_r4 RANKS=8 ZEST_SWARM_MIN_ROUNDS=4 && \
run r6t_n8_r2 RANKS=8 ZEST_SWARM_MIN_ROUNDS=2 && \
run r6t_n4_r4 RANKS=4 ZEST_SWARM_MIN_ROUNDS=4
