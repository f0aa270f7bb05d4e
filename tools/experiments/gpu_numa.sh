#!/bin/bash
# NUMA binding check on the GPU box: what sysfs says about the GPU, then the 1-GPU bench bound
# (default) and unbound (ZEST_NUMA_BIND=0).
mkdir -p gpurun_out/numa
timeout -k 10 120 python -c "
import os, torch
from zest_amd.parallel import gpu_local_cpus
d = torch.device('cuda', 0)
p = torch.cuda.get_device_properties(d)
print('bdf', hex(p.pci_domain_id), hex(p.pci_bus_id), hex(p.pci_device_id))
near = gpu_local_cpus(d); allowed = os.sched_getaffinity(0)
print('near', len(near), sorted(near)[:8], 'allowed', len(allowed), sorted(allowed)[:8], 'overlap', len(near & allowed))
" > gpurun_out/numa/info.log 2>&1 || exit $?
cat gpurun_out/numa/info.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/numa/bound.log 2>&1 || exit $?
grep -v '^{' gpurun_out/numa/bound.log; tail -1 gpurun_out/numa/bound.log | cut -c1-160
ZEST_NUMA_BIND=0 timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/numa/unbound.log 2>&1 || exit $?
tail -1 gpurun_out/numa/unbound.log | cut -c1-160
