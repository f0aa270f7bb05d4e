# round-5 call j: compressor v2 identity, origin adopted from the build's serialized store (setup),
# ipc host-wait, host-indexed decode row, concurrent pinning
set -o pipefail
mkdir -p gpurun_out/r5j
df -h /tmp . 2>/dev/null | tee gpurun_out/r5j/df.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "ser_store or device_puller or compress" > gpurun_out/r5j/kernels.log 2>&1 || { tail -30 gpurun_out/r5j/kernels.log; exit 1; }
tail -1 gpurun_out/r5j/kernels.log
STEPS=10 WARMUP=2 bash tools/gpu/check.sh r5j bench || exit 1
bash tools/gpu/check.sh r5j gpubench || exit 1
RANKS=2 bash tools/gpu/check.sh r5j rehearsal || exit 1
bash tools/gpu/check.sh r5j pin
