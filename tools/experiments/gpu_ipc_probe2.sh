#!/bin/bash
# Which condition makes the sibling-rank IPC import hang: arena size, NUMA binding, pinned memory?
mkdir -p gpurun_out/ipcp2
run() {
  timeout -k 10 120 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29571 tools/experiments/ipc_probe2.py "$@" > gpurun_out/ipcp2/$1_$2_$3.log 2>&1
  local rc=$?; echo "== $* rc=$rc"; grep -E "rank [01]:|Timeout|File" gpurun_out/ipcp2/$1_$2_$3.log | head -12; return $rc
}
run 16 plain 1 && run 16 plain 8
