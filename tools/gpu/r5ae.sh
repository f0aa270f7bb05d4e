# round-5 call ae: where the public path's first call goes (7-8 s on 70B against 2.6 s for later calls)
set -o pipefail
mkdir -p gpurun_out/r5ae
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
SR_MODEL=llama-3.1-70b SR_MODES=random bash tools/gpu/check.sh r5ae swarmrow || exit 1
tail -1 gpurun_out/r5ae/swarmrow.log | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print({k: e[k] for k in e if 'warm' in k or 'first' in k or 'setup' in k or k == 'swarm_pull_phases'})"
