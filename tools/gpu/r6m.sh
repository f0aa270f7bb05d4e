# round-6 call m: swarm GPU tests (event-ordered tables, windows, freed arenas); N = 1 bench (70B, engine + public row)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6m
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $PYT -v tests/test_gpu_device.py -k "swarm or refilled" > gpurun_out/r6m/swarm.log 2>&1; echo "swarm rc $?"; tail -1 gpurun_out/r6m/swarm.log
ZEST_SWARM_UNORDERED_TABLES=1 timeout -k 10 300 $PYT tests/test_gpu_device.py -k hash_table_ordered > gpurun_out/r6m/race_restored.log 2>&1; echo "race restored rc $? (expect 1)"; tail -1 gpurun_out/r6m/race_restored.log
bash tools/gpu/check.sh r6m bench
