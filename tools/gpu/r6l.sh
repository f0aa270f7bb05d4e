# round-6 call l: exchange windows (swarm GPU tests incl. freed arenas); 2/4/8-rank rehearsals;
# BG4 staging HBM writes (WRITE_SIZE of k_lz4_pair, staging on / off)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print('$1', d['value'], {k: e[k] for k in e if k in ('random_GBps','swarm_pull_GBps','swarm_pull_step_s','swarm_pull_error','swarm_pull_exchange')})"; }
mkdir -p gpurun_out/r6l
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $PYT -v tests/test_gpu_device.py -k "swarm or refilled" > gpurun_out/r6l/swarm.log 2>&1; echo "swarm rc $?"; grep -cE "PASSED" gpurun_out/r6l/swarm.log; tail -1 gpurun_out/r6l/swarm.log
for st in 1 0; do
  ZG_BG4_STAGE=$st timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r6l/wpmc_$st -o p --output-format csv -- \
    python3 -m zest_amd.gpubench --json --mib 256 --runs 2 > gpurun_out/r6l/wpmc_$st.log 2>&1 || { echo "wpmc $st failed"; break; }
  echo "BG4 staging $st:"; python tools/gpu/pmc_write.py gpurun_out/r6l/wpmc_$st --output-bytes 268435456
done
RANKS=2 bash tools/gpu/check.sh r6l_n2 rehearsal > /dev/null && show r6l_n2 && \
RANKS=4 bash tools/gpu/check.sh r6l_n4 rehearsal > /dev/null && show r6l_n4 && \
RANKS=8 bash tools/gpu/check.sh r6l_n8 rehearsal > /dev/null && show r6l_n8
