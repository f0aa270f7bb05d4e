# round-5 call o: GPU CLI after the no-wait-for-teardown change; staging 512 vs 256 MB; swarm_pull
# loopback trace (where the cache writes run) + N=1 public path from a loopback seeder
set -o pipefail
mkdir -p gpurun_out/r5o
CLI_MODE=bf16 bash tools/gpu/check.sh r5o clipeer || exit 1
CLI_MODE=bf16 CLIPEER_TAG=_st256 CLIPEER_GPU_ENV="ZEST_GPU_STAGING_MB=256" bash tools/gpu/check.sh r5o clipeer || exit 1
bash tools/gpu/check.sh r5o swarmtrace
