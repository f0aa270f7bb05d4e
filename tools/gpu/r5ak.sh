# round-5 call ak: 4-rank rehearsal on the one GPU (gloo control, VMM-mapped arenas) with GPU-side
# exchange readiness: 3 peers per rank, waits on several counters per exchange stream
set -o pipefail
mkdir -p gpurun_out/r5ak
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
RANKS=4 bash tools/gpu/check.sh r5ak rehearsal || exit 1
tail -1 gpurun_out/r5ak/rehearsal.log | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print({k: e[k] for k in e if 'signals' in k or 'wait' in k or 'GBps' in k or 'ms_per' in k})"
