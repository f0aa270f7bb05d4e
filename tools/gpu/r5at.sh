# round-5 call at: quarter-round staging default at N > 1: swarm GPU tests, 4-rank rehearsal
set -o pipefail
mkdir -p gpurun_out/r5at
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_device.py \
  -k "reuses_peer_mapped or swarm_pull" > gpurun_out/r5at/swarm.log 2>&1 || { tail -40 gpurun_out/r5at/swarm.log; exit 1; }
grep -cE "PASSED" gpurun_out/r5at/swarm.log
RANKS=4 bash tools/gpu/check.sh r5at rehearsal
