# round-6 call ff: HBM bytes written by k_lz4_pair at the final decoder (dynamic schedule, unrolled
# ungroup), BG4 staging on / off, and staged under the static schedule; 256 MiB of BG4 bf16 (gpubench)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6ff
for st in 1 0 1s; do
  export ZG_PAIR_DYNAMIC=1; [ "$st" = "1s" ] && export ZG_PAIR_DYNAMIC=0
  ZG_BG4_STAGE=${st%s} timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r6ff/wpmc_$st -o p --output-format csv -- \
    python3 -m zest_amd.gpubench --json --mib 256 --runs 2 > gpurun_out/r6ff/wpmc_$st.log 2>&1 || { echo "wpmc $st failed"; exit 1; }
  echo "BG4 staging ${st%s} (dynamic schedule $ZG_PAIR_DYNAMIC):"; python tools/gpu/pmc_write.py gpurun_out/r6ff/wpmc_$st --output-bytes 268435456
done
