# round-5 call u: peer-mapped arena + swarm GPU tests after the ipc-lag change; the public path on the
# 70B bf16 world (BG4-LZ4 decoded inside swarm_pull's device pipeline) next to the engine
set -o pipefail
mkdir -p gpurun_out/r5u
bash tools/gpu/check.sh r5u ipc swarm || exit 1
SR_MODEL=llama-3.1-70b SR_MODES=bf16 bash tools/gpu/check.sh r5u swarmrow
