# round-6 call nn: the parse's block loop restated wave-uniform + branch-free prefetch (SGPR spills
# 57 -> 42, VGPR spills 4 -> 16): decoder numerics tests, two split-probe runs, HBM bytes written,
# 256 MiB of BG4 bf16
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6nn
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r6nn/kernels.log 2>&1; rc=$?; echo "kernel tests rc $rc: $(tail -1 gpurun_out/r6nn/kernels.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/gpu/lz4_split_probe.py --mib 256 1024 --runs 10 > gpurun_out/r6nn/probe.log 2>&1 || { tail -5 gpurun_out/r6nn/probe.log; exit 1; }
timeout -k 10 300 python -u tools/gpu/lz4_split_probe.py --mib 256 1024 --runs 10 >> gpurun_out/r6nn/probe.log 2>&1 || exit 1
cut -c1-400 gpurun_out/r6nn/probe.log
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r6nn/wpmc -o p --output-format csv -- \
  python3 -m zest_amd.gpubench --json --mib 256 --runs 2 > gpurun_out/r6nn/wpmc.log 2>&1 || { echo "wpmc failed"; exit 1; }
python tools/gpu/pmc_write.py gpurun_out/r6nn/wpmc --output-bytes 268435456
