# round-5 call d: new device tests, config-2 rehearsal, swarm GPU tests, 70B headline bench + swarm row
set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 300 python -u -m pytest tests/test_gpu_device.py -x -v --timeout 120 --timeout-method thread \
  -k "sibling or second_gpu or pull_files_multi or direct_pull" > gpurun_out/r5d/devtests.log 2>&1 || { tail -30 gpurun_out/r5d/devtests.log; exit 1; }
tail -1 gpurun_out/r5d/devtests.log
STEPS=10 WARMUP=3 bash tools/gpu/check.sh r5d config2 swarm bench
