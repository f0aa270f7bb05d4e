# round-5 call m: the LZ4 pair decoder hashing what it decodes (ZG_FUSED_HASH): numerics, the 256 MiB
# ingest rows (fused vs not), the 70B bench
set -o pipefail
mkdir -p gpurun_out/r5m
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "decoder_hash or ingest or device_puller or bg4 or compress or lz4" > gpurun_out/r5m/kernels.log 2>&1 \
  || { tail -40 gpurun_out/r5m/kernels.log; exit 1; }
tail -1 gpurun_out/r5m/kernels.log
bash tools/gpu/check.sh r5m gpubench || exit 1
mkdir -p gpurun_out/r5m/nofuse
GPUBENCH_ENV="ZG_FUSED_HASH=0" bash tools/gpu/check.sh r5m/nofuse gpubench || exit 1
STEPS=5 WARMUP=2 bash tools/gpu/check.sh r5m bench
