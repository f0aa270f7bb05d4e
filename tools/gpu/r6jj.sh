# round-6 call jj: the parse prefetching its compressed stream into L2 through LDS-DMA loads (after the kernarg change, scratch
# 164 -> 36 B/lane): decoder numerics tests, the time split probe, and HBM bytes written (staged,
# dynamic schedule), 256 MiB of BG4 bf16
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6jj
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r6jj/kernels.log 2>&1; rc=$?; echo "kernel tests rc $rc: $(tail -1 gpurun_out/r6jj/kernels.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/gpu/lz4_split_probe.py --mib 256 1024 > gpurun_out/r6jj/probe.log 2>&1 || { tail -5 gpurun_out/r6jj/probe.log; exit 1; }
tail -2 gpurun_out/r6jj/probe.log
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r6jj/wpmc -o p --output-format csv -- \
  python3 -m zest_amd.gpubench --json --mib 256 --runs 2 > gpurun_out/r6jj/wpmc.log 2>&1 || { echo "wpmc failed"; exit 1; }
python tools/gpu/pmc_write.py gpurun_out/r6jj/wpmc --output-bytes 268435456
