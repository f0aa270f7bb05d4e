# round-5 call aq: automatic peer-mapped arena reuse: the new repeat test + the swarm GPU tests, then
# the full GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out/r5aq
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_device.py \
  -k "reuses_peer_mapped or swarm_pull" > gpurun_out/r5aq/swarm.log 2>&1 || { tail -40 gpurun_out/r5aq/swarm.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r5aq/swarm.log
bash tools/gpu/check.sh r5aq tests smoke
