# round-5 call ba: closing N = 1 check at HEAD: swarm GPU tests, smoke, driver-shaped bench (20 / 5)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
STEPS=20 WARMUP=5 bash tools/gpu/check.sh r5ba swarm smoke bench || exit 1
