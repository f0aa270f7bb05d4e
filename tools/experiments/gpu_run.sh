export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 240 python tools/kbench.py --gib 4 > gpurun_out/kbench.log 2>&1; rc=$?; echo "kbench rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --model llama-3.1-8b --steps 3 --warmup 1 > gpurun_out/bench8b.log 2>&1; rc=$?; echo "bench8b rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench70b.log 2>&1; echo "bench70b rc=$?"
