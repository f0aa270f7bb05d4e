mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "index_scan or ingest_matches_cpu or ingest_detects or real_hf_xet or device_puller" > gpurun_out/r5c/kernel_tests.log 2>&1 && \
timeout -k 10 300 python -u -m zest_amd.gpubench --json --mib 256 --runs 7 > gpurun_out/r5c/gpubench256.json 2> gpurun_out/r5c/gpubench256.err && \
timeout -k 10 500 python -u bench.py --model llama-3.1-8b --steps 5 --warmup 2 --swarm-steps 3 > gpurun_out/r5c/bench8b.log 2>&1
