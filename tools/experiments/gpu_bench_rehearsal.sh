#!/bin/bash
# Multi-rank bench.py rehearsal on a one-GPU box: 2 ranks share the GPU over gloo and replicate
# through gloo collectives on device tensors (EXCHANGES, default "bcast allgather"; the peer-mapped
# ipc / xgmi modes hung in hipIpcOpenMemHandle here with 16 GB arenas), Llama-3.1-8B.
export ZEST_SKIP_BUILD=1 ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 ZEST_BENCH_WATCHDOG=150
mkdir -p gpurun_out/rehearsal
for ex in ${EXCHANGES:-bcast allgather}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29561 bench.py --gpus 2 --model llama-3.1-8b --exchange $ex --steps 2 --warmup 1 \
      > gpurun_out/rehearsal/$ex.log 2>&1 || { grep -v amdgpu.ids gpurun_out/rehearsal/$ex.log | tail -80; exit 1; }
  grep "^\[bench" gpurun_out/rehearsal/$ex.log
  tail -1 gpurun_out/rehearsal/$ex.log | cut -c1-400
done
