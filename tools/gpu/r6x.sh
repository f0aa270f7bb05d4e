# round-6 call x: swarm GPU tests + the 8-rank rehearsal again (r6w's row fell to 0.37-0.48 of the
# engine), with per-item layout buffers reused; dynamic decoder schedule on vs off
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']
print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k in ('swarm_pull_step_s',)})
print('   rank0 threads', (e.get('swarm_pull_thread_cpu_s') or [None])[0])"; }
run() { tag=$1; shift; env "$@" bash tools/gpu/check.sh $tag rehearsal > /dev/null && show $tag; }
export REHEARSAL_ARGS="--swarm-steps 3"
mkdir -p gpurun_out/r6x
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_device.py -k "swarm" > gpurun_out/r6x/swarm.log 2>&1; rc=$?; echo "swarm tests rc $rc: $(tail -1 gpurun_out/r6x/swarm.log)"; [ $rc = 0 ] && \
run r6x_n8 RANKS=8 && \
run r6x_n8_static RANKS=8 ZG_PAIR_DYNAMIC=0
