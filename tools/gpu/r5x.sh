# round-5 call x: the device pull copies only the fetched runs (not the reserved holes between them):
# full GPU suite, then the public path on the 70B bf16 world with the new copies and with the old
# whole-span copy (ZEST_H2D_WHOLE_SPAN=1), same box
set -o pipefail
mkdir -p gpurun_out/r5x/old
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
bash tools/gpu/check.sh r5x tests || exit 1
SR_MODEL=llama-3.1-70b SR_MODES=bf16 bash tools/gpu/check.sh r5x swarmrow || exit 1
ZEST_H2D_WHOLE_SPAN=1 SR_MODEL=llama-3.1-70b SR_MODES=bf16 bash tools/gpu/check.sh r5x/old swarmrow
for f in gpurun_out/r5x/swarmrow.log gpurun_out/r5x/old/swarmrow.log; do
  tail -1 $f | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print(sys.argv[1], e.get('swarm_pull_GBps'), e.get('swarm_pull_device_timeline'))" $f
done
