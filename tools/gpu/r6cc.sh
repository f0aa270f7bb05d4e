# round-6 call cc: the pull pipeline's streams at the device's greatest priority (the engine's
# split) vs normal priority, 8-rank and 4-rank rehearsals, both data modes; swarm GPU tests first
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('$1', {k: e[k] for k in e if k.endswith(('_vs_engine','_error')) or k in ('swarm_pull_step_s',)})"; }
mkdir -p gpurun_out/r6cc
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_device.py -k "swarm" > gpurun_out/r6cc/swarm.log 2>&1; rc=$?; echo "swarm tests rc $rc: $(tail -1 gpurun_out/r6cc/swarm.log)"; [ $rc = 0 ] || exit 1
run() { tag=$1; shift; env "$@" bash tools/gpu/check.sh $tag rehearsal > /dev/null && show $tag; }
export REHEARSAL_ARGS="--swarm-steps 3"
run r6cc_n8_hi RANKS=8 && \
run r6cc_n8_normal RANKS=8 ZEST_PULL_STREAM_PRIORITY=0 && \
run r6cc_n4_hi RANKS=4
