# round-5 call ay: 8 ranks on the one GPU, 5 timed public-path pulls each: 512 MiB (half-round)
# staging slots, then 256 MiB again -- does a half round keep the gain without the ~2.5 s stall?
set -o pipefail
export SW_ARGS="--swarm-steps 5"
sed -n '/^run()/,/^}/p' tools/gpu/r5av.sh | sed 's/--swarm-steps 3 //' > /tmp/run_fn.sh
mkdir -p gpurun_out/r5av
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp ZEST_BENCH_BACKEND=gloo
source /tmp/run_fn.sh
run ${RUNS_A:-n8_512_s5} ZEST_SWARM_STAGING_MB=${MB_A:-512} && run ${RUNS_B:-n8_256_s5} ZEST_SWARM_STAGING_MB=${MB_B:-256}
