# round-5 call p: GPU suite after the deferred cache copies; swarm_pull loopback trace (fetch threads
# free of cache work) + public path N=1/2 from a loopback seeder; GPU CLI vs host (bf16, random)
set -o pipefail
mkdir -p gpurun_out/r5p
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5p/tests.log 2>&1 || { tail -40 gpurun_out/r5p/tests.log; exit 1; }
tail -1 gpurun_out/r5p/tests.log
bash tools/gpu/check.sh r5p swarmtrace || exit 1
SWARM_RANKS=1,2 bash tools/gpu/check.sh r5p swarmbench || exit 1
CLI_MODE=bf16 bash tools/gpu/check.sh r5p clipeer || exit 1
CLI_MODE=random bash tools/gpu/check.sh r5p clipeer
