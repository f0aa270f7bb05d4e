# round-6 closing run at the final tree: full GPU test suite, smoke, and the driver's N = 1 bench
# (--steps 20 --warmup 5)
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
bash tools/gpu/check.sh ${TAG:-r6final} tests smoke && \
STEPS=20 WARMUP=5 bash tools/gpu/check.sh ${TAG:-r6final} bench > /dev/null && \
grep '^{"metric' gpurun_out/${TAG:-r6final}/bench.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('bench', d['value'], d['ms_per_step'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine'))})"
