# round-6 call u: what bounds k_lz4_pair at 256 MiB vs 1 GiB (SQ counters: scalar / vector issue,
# scalar-memory instructions, waits); random-mode rows with 4 rounds per share at 4 / 8 ranks;
# 8 GB stripe with the fdatasync span
set -o pipefail
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r6u
for mib in 256 1024; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE \
    --kernel-trace -d gpurun_out/r6u/pmcA_$mib -o p --output-format csv -- python3 -m zest_amd.gpubench --json --mib $mib --runs 2 > gpurun_out/r6u/pmcA_$mib.log 2>&1 || { echo "pmcA $mib failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_WAIT_ANY GRBM_COUNT \
    --kernel-trace -d gpurun_out/r6u/pmcB_$mib -o p --output-format csv -- python3 -m zest_amd.gpubench --json --mib $mib --runs 2 > gpurun_out/r6u/pmcB_$mib.log 2>&1 || { echo "pmcB $mib failed"; exit 1; }
  python tools/gpu/pmc_table.py gpurun_out/r6u/pmcA_$mib gpurun_out/r6u/pmcB_$mib --raw gpurun_out/r6u/raw_$mib.json > gpurun_out/r6u/table_$mib.md && \
  python - $mib <<'PY'
import json, sys
mib = sys.argv[1]
raw = json.load(open(f"gpurun_out/r6u/raw_{mib}.json"))
for k, c in raw.items():
    if "k_lz4_pair" in k:
        print(mib, k.split("(")[0][:40], {n: round(v) for n, v in sorted(c.items())})
PY
done
show() { grep '^{"metric' gpurun_out/$1/rehearsal.log | tail -1 | python -c "
import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']
print('$1', d['value'], {k: e[k] for k in e if k.endswith(('_GBps','_vs_engine','_error')) or k == 'swarm_pull_step_s'})"; }
run() { tag=$1; shift; env "$@" bash tools/gpu/check.sh $tag rehearsal > /dev/null && show $tag; }
export REHEARSAL_ARGS="--modes random --swarm-steps 3 --swarm-warmup 2"
run r6u_n4_r4 RANKS=4 ZEST_SWARM_MIN_ROUNDS=4 && \
run r6u_n8_r4 RANKS=8 ZEST_SWARM_MIN_ROUNDS=4 && \
STRIPE_MB=8192 bash tools/gpu/check.sh r6u_stripe stripe && python -c "
import json; d=json.load(open('gpurun_out/r6u_stripe/stripe.json'))
for k in ('1_seeder','3_seeders'): print(k, d[k]['seconds'], d[k].get('transfer_s'), d[k].get('cpu_s'), {x: d[k]['span_ms'].get(x) for x in ('download/fdatasync','download/pwrite','cache/put_pending')})"
