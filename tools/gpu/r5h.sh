# round-5 call h: timeline test, 70B public-path row with device timeline, striping (capped / uncapped),
# GPU CLI vs host CLI, counter table
set -o pipefail
mkdir -p gpurun_out/r5h
timeout -k 10 200 python -u -m pytest tests/test_gpu_device.py -x -q --timeout 120 --timeout-method thread \
  -k "sibling" > gpurun_out/r5h/timeline_test.log 2>&1 || { tail -30 gpurun_out/r5h/timeline_test.log; exit 1; }
tail -1 gpurun_out/r5h/timeline_test.log
SR_MODEL=llama-3.1-70b SR_MODES=random bash tools/gpu/check.sh r5h swarmrow || exit 1
STRIPE_ARGS="--rate-mbps 1250" bash tools/gpu/check.sh r5h/capped stripe || exit 1
bash tools/gpu/check.sh r5h/uncapped stripe || exit 1
bash tools/gpu/check.sh r5h cli pmctable
