# round-5 call ai: checkpoint at the late-round code (host decoder, merge gap, parallel walk, GPU-side
# readiness): full GPU suite, smoke, the driver-shaped bench (20 timed steps, 5 warm-up)
set -o pipefail
mkdir -p gpurun_out/r5ai
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
STEPS=20 WARMUP=5 bash tools/gpu/check.sh r5ai tests smoke bench
