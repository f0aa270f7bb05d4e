# round-6 call k: BG4 staged decode (kernel tests, gpubench rows); exchange windows (swarm GPU tests incl.
# freed arenas); 2/4/8-rank rehearsals
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error','swarm_pull_exchange')})"; }
mkdir -p gpurun_out/r6k
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
bash tools/gpu/check.sh r6k kernels && \
timeout -k 10 300 python -u -m zest_amd.gpubench --json > gpurun_out/r6k/gpubench_stage.json 2> gpurun_out/r6k/gpubench_stage.log && \
ZG_BG4_STAGE=0 timeout -k 10 300 python -u -m zest_amd.gpubench --json > gpurun_out/r6k/gpubench_nostage.json 2> gpurun_out/r6k/gpubench_nostage.log && \
python -c "
import json
for f in ('stage','nostage'):
    rows = {r['name']: round(r['throughput_mbps']/1e3, 1) for r in json.load(open(f'gpurun_out/r6k/gpubench_{f}.json'))['results']}
    print(f, {k: v for k, v in rows.items() if 'lz4' in k or 'ingest' in k})
" && \
timeout -k 10 600 $PYT -v tests/test_gpu_device.py -k "swarm or refilled" > gpurun_out/r6k/swarm.log 2>&1 && grep -cE "PASSED" gpurun_out/r6k/swarm.log && tail -1 gpurun_out/r6k/swarm.log && \
RANKS=2 bash tools/gpu/check.sh r6k_n2 rehearsal > /dev/null && show r6k_n2 && \
RANKS=4 bash tools/gpu/check.sh r6k_n4 rehearsal > /dev/null && show r6k_n4 && \
RANKS=8 bash tools/gpu/check.sh r6k_n8 rehearsal > /dev/null && show r6k_n8
