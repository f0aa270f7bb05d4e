# round-6 call ee: host striping, 1 vs 3 uncapped loopback seeders, 8 GB, with every cache and
# snapshot in memory (TMPDIR=/dev/shm): the receiver without the disk
set -o pipefail
export ZEST_SKIP_BUILD=1
mkdir -p gpurun_out/r6ee
for j in 16 48; do
  TMPDIR=/dev/shm timeout -k 10 600 python -u tools/stripe_bench.py --mb 8192 --jobs $j --trace /dev/shm/stripe_trace_$j \
    --out gpurun_out/r6ee/stripe_shm_j$j.json > gpurun_out/r6ee/stripe_shm_j$j.log 2>&1 || { echo "stripe j$j failed"; tail -5 gpurun_out/r6ee/stripe_shm_j$j.log; rm -rf /dev/shm/stripe_trace_$j /dev/shm/zest-stripe-*; exit 1; }
  rm -rf /dev/shm/stripe_trace_$j
  python -c "
import json; d=json.load(open('gpurun_out/r6ee/stripe_shm_j$j.json'))
print('j$j', 'speedup', d['speedup_3_vs_1'], 'transfer', d.get('transfer_speedup_3_vs_1'))
for k in ('1_seeder','3_seeders'): print('  ', k, d[k]['seconds'], d[k]['GBps'], d[k].get('transfer_s'), d[k].get('cpu_s'), d[k].get('cpus_busy'))"
done
rm -rf /dev/shm/zest-stripe-* 2>/dev/null; true
