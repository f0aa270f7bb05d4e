# round-5 call l: the full GPU suite + smoke at the current tree
set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5l/tests.log 2>&1 || { tail -40 gpurun_out/r5l/tests.log; exit 1; }
tail -2 gpurun_out/r5l/tests.log
bash tools/gpu/check.sh r5l smoke
