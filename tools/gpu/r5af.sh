# round-5 call af: public path on the 70B random world, runs merged across gaps <= 1 MiB (default:
# the terms' 0.8 % worst-case slack crosses PCIe) vs merged only when touching (ZEST_H2D_MERGE_GAP=0)
set -o pipefail
mkdir -p gpurun_out/r5af/gap0
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
SR_MODEL=llama-3.1-70b SR_MODES=random bash tools/gpu/check.sh r5af swarmrow || exit 1
ZEST_H2D_MERGE_GAP=0 SR_MODEL=llama-3.1-70b SR_MODES=random bash tools/gpu/check.sh r5af/gap0 swarmrow || exit 1
for f in gpurun_out/r5af/swarmrow.log gpurun_out/r5af/gap0/swarmrow.log; do
  tail -1 $f | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print(sys.argv[1], e['random_GBps'], e['swarm_pull_GBps'], e['swarm_pull_device_timeline'])" $f
done
