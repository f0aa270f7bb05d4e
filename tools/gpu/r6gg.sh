set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6gg
ZG_BG4_STAGE=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r6gg/wpmc -o p --output-format csv -- \
  python3 -m zest_amd.gpubench --json --mib 256 --runs 2 > gpurun_out/r6gg/wpmc.log 2>&1 || { echo "wpmc failed"; exit 1; }
echo "decoder at c69c6e9, staged:"; python tools/gpu/pmc_write.py gpurun_out/r6gg/wpmc --output-bytes 268435456
