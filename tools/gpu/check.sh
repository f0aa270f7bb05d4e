#!/bin/bash
# GPU-box measurement steps, run through gpurun from this container:
#
#   gpurun --timeout 1100 -- 'bash tools/gpu/check.sh OUT_DIR step [step ...]'
#
# Every step runs under its own time limit; the first step that fails, times out or faults ends the
# script (nothing more touches the GPU after it).  Logs land in gpurun_out/OUT_DIR/.
#
# steps:
#   kernels     HIP kernel numerics tests (tests/test_gpu_kernels.py)
#   tests       full `pytest -m gpu` (one process)
#   smoke       __graft_entry__.smoke()
#   bench       default `python bench.py` (N=1, Llama-3.1-70B, bf16 headline + random) ($STEPS/$WARMUP)
#   rehearsal   self-launched `bench.py --gpus $RANKS` (default 2) on the one GPU (gloo control, ranks
#               share the device; --exchange auto incl. the VMM-mapped ipc/xgmi modes), Llama-3.1-8B
#   ipc         peer-mapped arena tests (tests/test_gpu_ipc.py)
#   cli         `zest pull --gpus 1` vs host `zest pull` (Llama-3.1-8B from an HBM seeder, sync between)
#   stripe      host pull from 1 vs 3 loopback seeders
#   clipeer     `zest pull --gpus 1` vs host pull from warm `zest serve` seeders (tools/cli_peer_bench.py)
#   pin         $PIN_PROCS processes pinning $PIN_GB GB each at once (the N=8 origin setup)
#   seed        HBM seeding throughput (Mixtral-8x7B, chunks_served/s)
#   kbench      per-kernel micro-benchmarks ($KBENCH_ONLY selects one group, e.g. k3pair)
#   prof        rocprofv3 --kernel-trace --stats of the 70B bench -> per-kernel summary (markdown)
#   kprof       rocprofv3 --kernel-trace --stats of kbench ($KBENCH_ONLY) -> per-kernel summary
#   kvar        kbench ($KBENCH_ONLY) once per kernel-build variant in $VARIANTS (dirs under variants/, each a
#               zest_amd package copy with its own _hip .so) -> kbench_<variant>.jsonl
#   kpmc        rocprofv3 --pmc SQ counters (per launch) of kbench ($KBENCH_ONLY), kernels matching $PMC_KERNEL
#   swarmtrace  public pull(device="all") at N = 1 under ZEST_TRACE (Chrome trace of the device pipeline:
#               fetch waits, H2D + decode/hash submits, settle) -> trace summary
#   hostbench   `zest bench --synthetic` on the box's CPU
#   benchA/benchB  bench.py --modes $BENCH_MODES (bf16) with extra env $BENCH_ENV_A / $BENCH_ENV_B (A/B of opt-ins)
#   gpubench    `zest bench --gpu --json` rows ($GPUBENCH_ENV: extra env, e.g. "ZG_LZ4_PAIR=0")
#   swarm       term-sharded swarm_pull GPU tests (modes, VMM fault hooks) (tests/test_gpu_device.py -k swarm_pull)
#   swarmbench  public pull(device="all") end to end from a loopback HBM seeder, $SWARM_RANKS (1,2,3) ranks,
#               $SWARM_MODEL (llama-3.1-8b) -> swarm_pull.json
set -o pipefail
OUT=gpurun_out/${1:?usage: check.sh OUT_DIR step...}
shift
mkdir -p "$OUT"
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
STEPS=${STEPS:-5}
WARMUP=${WARMUP:-2}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"

fail() { echo "[check] step $1 failed (rc=$2)"; tail -40 "$3" | grep -v amdgpu.ids; exit 1; }

for step in "$@"; do
  log=$OUT/$step.log
  t0=$(date +%s)
  case $step in
    kernels) timeout -k 10 400 $PYT tests/test_gpu_kernels.py > $log 2>&1 || fail $step $? $log
             tail -1 $log ;;
    tests) timeout -k 10 1000 $PYT -m gpu tests > $log 2>&1 || fail $step $? $log
           tail -1 $log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || fail $step $? $log
           grep -h "smoke" $log ;;
    bench) timeout -k 10 900 python -u bench.py --steps $STEPS --warmup $WARMUP > $log 2>&1 || fail $step $? $log
           grep -h "aggregate" $log; tail -1 $log | cut -c1-400 ;;
    rehearsal) ZEST_BENCH_BACKEND=gloo ZEST_BENCH_LOG_ALL=1 timeout -k 10 700 python -u bench.py --gpus ${RANKS:-2} \
                 --model llama-3.1-8b --steps 3 --warmup 1 ${REHEARSAL_ARGS:-} > $log 2>&1 || fail $step $? $log
               grep -h "mapped\|autotune\|GB/s aggregate" $log | head -12; tail -1 $log | cut -c1-600 ;;
    ipc) timeout -k 10 400 $PYT -v tests/test_gpu_ipc.py > $log 2>&1 || fail $step $? $log
         grep -E "PASSED|FAILED|SKIPPED" $log ;;
    cli) timeout -k 10 700 python -u tools/direct_bench.py --model llama-3.1-8b --skip-direct --host-after \
           --mode ${CLI_MODE:-random} --out $OUT/cli_vs_host_${CLI_MODE:-random}.json > $log 2>&1 || fail $step $? $log
         grep -h "^\[" $log ;;
    clipeer) timeout -k 10 900 python -u tools/cli_peer_bench.py --mb ${CLIPEER_MB:-8192} --mode ${CLI_MODE:-bf16} \
               --seeders ${CLIPEER_SEEDERS:-1} --gpu-env "${CLIPEER_GPU_ENV:-}" \
               --out $OUT/cli_peer_${CLI_MODE:-bf16}${CLIPEER_TAG:-}.json > $log 2>&1 || fail $step $? $log
             grep -h "^\[" $log ;;
    pin) timeout -k 10 500 python -u tools/pin_bench.py --procs ${PIN_PROCS:-8} --gb ${PIN_GB:-17.6} \
           --out $OUT/pin_${PIN_PROCS:-8}x${PIN_GB:-17.6}.json > $log 2>&1 || fail $step $? $log
         tail -1 $log | cut -c1-400 ;;
    stripe) mkdir -p $OUT/stripe_trace
            timeout -k 10 600 python -u tools/stripe_bench.py --mb ${STRIPE_MB:-4096} ${STRIPE_ARGS:-} \
              --trace $OUT/stripe_trace --out $OUT/stripe.json > $log 2>&1 \
              || fail $step $? $log
            grep -h "^\[" $log; rm -rf $OUT/stripe_trace ;;
    seed) timeout -k 10 600 python -u tools/seed_bench.py > $log 2>&1 || fail $step $? $log
          tail -5 $log ;;
    kbench) timeout -k 10 600 python -u tools/kbench.py ${KBENCH_ONLY:+--only $KBENCH_ONLY} > $OUT/kbench.jsonl 2> $log \
              || fail $step $? $log
            grep -h kernel $OUT/kbench.jsonl | cut -c1-200 ;;
    prof) timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o b70 -- \
            python3 bench.py --steps 3 --warmup 1 > $log 2>&1 || fail $step $? $log
          db=$(find $OUT/prof -name "*.db" | head -1)
          python tools/rocpd_summary.py "$db" --title "70B bench kernels ($(git log -1 --format=%h 2>/dev/null || echo tree))" \
            > $OUT/kernels.md 2>&1
          head -30 $OUT/kernels.md; rm -f "$db" ;;
    kprof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kprof -o kb -- \
             python3 tools/kbench.py ${KBENCH_ONLY:+--only $KBENCH_ONLY} > $log 2>&1 || fail $step $? $log
           db=$(find $OUT/kprof -name "*.db" | head -1)
           python tools/rocpd_summary.py "$db" --title "kbench ${KBENCH_ONLY:-all} kernels" > $OUT/kernels_kbench.md 2>&1
           head -24 $OUT/kernels_kbench.md; rm -f "$db" ;;
    gprof) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/gprof -o gb -- \
             python3 -m zest_amd.gpubench --json --mib ${GPROF_MIB:-256} --runs 5 > $log 2>&1 || fail $step $? $log
           db=$(find $OUT/gprof -name "*.db" | head -1)
           python tools/rocpd_summary.py "$db" --title "gpubench ${GPROF_MIB:-256} MiB kernels" > $OUT/kernels_gpubench.md 2>&1
           head -30 $OUT/kernels_gpubench.md; rm -f "$db" ;;
    benchA|benchB) v=BENCH_ENV_${step#bench}; env ${!v:-} timeout -k 10 700 python -u bench.py --modes ${BENCH_MODES:-bf16} \
                --steps $STEPS --warmup $WARMUP > $log 2>&1 || fail $step $? $log
              echo "env: ${!v:-}"; grep -h "aggregate" $log ;;
    gpubench) env ${GPUBENCH_ENV:-} timeout -k 10 500 python -u -m zest_amd.gpubench --json > $OUT/gpubench.json 2> $log \
                || fail $step $? $log
              python -c "import json,sys; [print(r['name'], round(r['throughput_mbps']/1e3,1), 'GB/s') for r in json.load(open(sys.argv[1]))['results']]" $OUT/gpubench.json ;;
    swarm) timeout -k 10 500 $PYT -v -s tests/test_gpu_device.py -k swarm_pull > $log 2>&1 || fail $step $? $log
           grep -E "PASSED|FAILED|^\[swarm_pull" $log ;;
    swarmbench) timeout -k 10 700 python -u tools/swarm_bench.py --model ${SWARM_MODEL:-llama-3.1-8b} \
                  --ranks ${SWARM_RANKS:-1,2,3} ${SWARM_ARGS:-} --out $OUT/swarm_pull.json > $log 2>&1 || fail $step $? $log
                grep -h "^\[" $log ;;
    kvar) for v in ${VARIANTS:?}; do
            ZEST_PKG_ROOT=variants/$v timeout -k 10 300 python -u tools/kbench.py ${KBENCH_ONLY:+--only $KBENCH_ONLY} \
              > $OUT/kbench_$v.jsonl 2>> $log || fail $step $? $log
            echo "variant $v"; grep -h '"kernel"' $OUT/kbench_$v.jsonl | cut -c1-110
          done ;;
    kpmc) timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
            SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVES --kernel-trace -d $OUT/pmc -o p \
            --output-format csv -- python3 tools/kbench.py ${KBENCH_ONLY:+--only $KBENCH_ONLY} > $log 2>&1 \
            || fail $step $? $log
          f=$(find $OUT/pmc -name "*counter_collection.csv" | head -1)
          python tools/gpu/pmc_summary.py "$f" "${PMC_KERNEL:-lz4}" > $OUT/pmc_summary.txt 2>&1; cat $OUT/pmc_summary.txt
          rm -rf $OUT/pmc ;;
    copytrace) # public-path swarm row under kernel + memory-copy + marker traces: does H2D overlap ingest?
               ZEST_BENCH_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace \
                 -d $OUT/ct -o ct -- python3 bench.py --model ${CT_MODEL:-llama-3.1-8b} \
                 --modes ${CT_MODES:-random} --steps 2 --warmup 1 --swarm-steps 2 --swarm-warmup 1 > $log 2>&1 \
                 || fail $step $? $log
               grep -h "aggregate" $log
               python tools/gpu/overlap.py $OUT/ct --between spin_kernel > $OUT/overlap_swarm.txt 2>&1
               python tools/gpu/overlap.py $OUT/ct > $OUT/overlap_all.txt 2>&1
               python tools/gpu/copy_rates.py $OUT/ct > $OUT/copy_rates.txt 2>&1
               cat $OUT/overlap_swarm.txt $OUT/overlap_all.txt $OUT/copy_rates.txt; rm -rf $OUT/ct ;;
    config2) # BASELINE config 2 on the public path: rank 0 warm, rank 1 cold, ranks share the GPU (gloo)
             ZEST_BENCH_BACKEND=gloo timeout -k 10 600 python -u tools/config2_rehearsal.py \
               --model ${C2_MODEL:-llama-3.1-8b} --mode ${C2_MODE:-bf16} --ranks ${C2_RANKS:-2} \
               --out $OUT/config2.json > $log 2>&1 || fail $step $? $log
             python -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in ('aggregate_GBps','leecher_receive_GBps','cdn_bytes','backend')}, [(r['rank'], r['exchange'], r['from_cache'], r['received_bytes'], r['pull_s']) for r in d['per_rank']])" $OUT/config2.json ;;
    swarmrow) timeout -k 10 600 python -u bench.py --model ${SR_MODEL:-llama-3.1-8b} --modes ${SR_MODES:-bf16,random} \
                --steps 5 --warmup 2 --swarm-steps 3 > $log 2>&1 || fail $step $? $log
              grep -h "GB/s aggregate\|swarm_pull" $log | cut -c1-300 ;;
    pmctable) # one counter group per rocprofv3 pass (SQ <= 8, TCC <= 4: FETCH_SIZE uses 3, WRITE_SIZE 2)
              i=0
              for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
                         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
                         "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT TCC_MISS"; do
                i=$((i+1))
                timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $OUT/pmc_$i -o p --output-format csv -- \
                  python3 -m zest_amd.gpubench --json --mib ${PMC_MIB:-256} --runs 2 > $log.$i 2>&1 || fail $step $? $log.$i
                timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $OUT/pmc_$i -o g --output-format csv -- \
                  python3 tools/kbench.py --only gather --iters 2 >> $log.$i 2>&1 || fail $step $? $log.$i
              done
              python tools/gpu/pmc_table.py $OUT/pmc_1 $OUT/pmc_2 $OUT/pmc_3 $OUT/pmc_4 --raw $OUT/pmc_raw.json \
                > $OUT/pmc_table.md 2>&1
              cat $OUT/pmc_table.md; rm -rf $OUT/pmc_? ;;
    swarmtrace) ZEST_TRACE=$PWD/$OUT/swarm_trace.%p.json timeout -k 10 400 python -u tools/swarm_bench.py \
                  --model ${SWARM_MODEL:-llama-3.1-8b} --ranks 1 --out $OUT/swarm_trace_run.json > $log 2>&1 \
                  || fail $step $? $log
                grep -h "^\[N=" $log | cut -c1-200
                for t in $OUT/swarm_trace.*.json; do echo "== $t"; python tools/trace_summary.py $t --top 20; done \
                  > $OUT/swarm_trace_summary.txt 2>&1
                cat $OUT/swarm_trace_summary.txt; rm -f $OUT/swarm_trace.*.json ;;
    hostbench) ./zest_amd/_bin/zest bench --synthetic > $log 2>&1 || fail $step $? $log
               lscpu | grep -E "Model name|^CPU\(s\)" >> $log; cat $log ;;
    *) echo "[check] unknown step $step"; exit 2 ;;
  esac
  echo "[check] $step ok in $(( $(date +%s) - t0 ))s"
done
