# round-6 call v: k_lz4_pair time split (parse alone vs the whole launch; largest vs smallest quarter
# of the chunks) at 256 MiB and 1 GiB; the decoder numerics tests after the kernel's new argument
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6v
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r6v/kernels.log 2>&1; rc=$?; echo "kernel tests rc $rc: $(tail -1 gpurun_out/r6v/kernels.log)"; [ $rc = 0 ] && \
timeout -k 10 300 python -u tools/gpu/lz4_split_probe.py --mib 256 1024 > gpurun_out/r6v/probe.log 2>&1; rc=$?; cat gpurun_out/r6v/probe.log | tail -4; exit $rc
