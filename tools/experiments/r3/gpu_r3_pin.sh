#!/bin/bash
# Round 3: pinned-host allocation / D2H / pwrite-source probe; then IPC import size threshold
# (2 ranks on the one GPU: 64 MiB, 512 MiB fresh arenas; stop at the first hang).
OUT=gpurun_out/r3pin; mkdir -p $OUT
export ZEST_SKIP_BUILD=1 IPC_PROBE_TIMEOUT=25
hipcc -O2 --offload-arch=gfx950 -o $OUT/pinned_probe tools/experiments/pinned_probe.cpp || exit 1
timeout -k 10 120 $OUT/pinned_probe /tmp > $OUT/pinned_probe.txt 2>&1 || { cat $OUT/pinned_probe.txt; exit 1; }
cat $OUT/pinned_probe.txt
rm -f $OUT/pinned_probe
port=29591
for cfg in "0.0625 plain 0 plain" "0.5 plain 0 plain"; do
  set -- $cfg
  port=$((port+1))
  timeout -k 5 45 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port $port tools/experiments/ipc_probe2.py $cfg > $OUT/ipc_$1_$4.log 2>&1
  rc=$?
  echo "cfg [$cfg] rc=$rc"; grep -h "imported\|rank .: ok\|Timeout" $OUT/ipc_$1_$4.log | head -4
  if [ $rc -ne 0 ]; then echo "case failed or hung: stop"; exit 0; fi
done
