# round-5 call aw: 8 ranks, 256 MiB staging, two warm-up pulls: is the slow first timed pull a
# second-call effect?
set -o pipefail
export SW_ARGS="--swarm-warmup 2"
sed -n '/^run()/,/^}/p' tools/gpu/r5av.sh > /tmp/run_fn.sh
mkdir -p gpurun_out/r5av
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp ZEST_BENCH_BACKEND=gloo
source /tmp/run_fn.sh
run n8_256_w2 ZEST_SWARM_STAGING_MB=256
