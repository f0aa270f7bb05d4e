#!/bin/bash
# Device-direct pull (Llama-3.1-8B from an HBM seeder over loopback): connections x fetch threads.
export ZEST_SKIP_BUILD=1 ZEST_CACHE_WRITES=0
mkdir -p gpurun_out/dsweep
for cfg in ${CFGS:-16:16 32:32 32:48}; do  # connections:threads
  set -- ${cfg/:/ }
  ZEST_PEER_CONNECTIONS=$1 timeout -k 10 300 python tools/direct_bench.py --model llama-3.1-8b --skip-host --skip-gpu-cli --threads $2 --out gpurun_out/dsweep/c$1_t$2.json > gpurun_out/dsweep/c$1_t$2.log 2>&1 || exit $?
  echo "conns=$1 threads=$2: $(grep -o '"direct_gbps": [0-9.]*' gpurun_out/dsweep/c$1_t$2.json) $(grep -o '"direct_nocache_gbps": [0-9.]*' gpurun_out/dsweep/c$1_t$2.json)"
done
