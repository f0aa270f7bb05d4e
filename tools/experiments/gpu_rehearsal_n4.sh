export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/reh4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 ZEST_BENCH_WATCHDOG=280
timeout -k 10 330 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29563 bench.py --gpus 4 --model llama-3.1-8b --exchange auto --steps 2 --warmup 1 \
  > gpurun_out/reh4/rehearsal_n4.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/reh4/rehearsal_n4.log | tail -12 | cut -c1-400; exit $rc
