# round-5 call aj: the public path's first call after the engine spent 4.5 s allocating its arena
# (two-mode bench); free memory + allocation time at that point, and a bare allocate/free/allocate probe
set -o pipefail
mkdir -p gpurun_out/r5aj
export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
timeout -k 10 300 python -u -c "
import time, torch
d = torch.device('cuda:0')
for i in range(3):
    f0 = torch.cuda.mem_get_info(d)[0]
    t = time.perf_counter(); x = torch.empty(141 << 30, dtype=torch.uint8, device=d); torch.cuda.synchronize(); ta = time.perf_counter() - t
    t = time.perf_counter(); x.fill_(1); torch.cuda.synchronize(); tf = time.perf_counter() - t
    del x; t = time.perf_counter(); torch.cuda.empty_cache(); te = time.perf_counter() - t
    print(f'[probe] round {i}: free {f0/1e9:.1f} GB, alloc {ta:.3f} s, first write {tf:.3f} s, empty_cache {te:.3f} s', flush=True)
" > gpurun_out/r5aj/alloc_probe.log 2>&1 || { tail -20 gpurun_out/r5aj/alloc_probe.log; exit 1; }
grep probe gpurun_out/r5aj/alloc_probe.log
bash tools/gpu/check.sh r5aj bench || exit 1
grep '^{' gpurun_out/r5aj/bench.log | tail -1 | python -c "import json,sys; d=json.JSONDecoder().raw_decode(sys.stdin.read())[0]; e=d['extra']; print({k: e[k] for k in e if 'first' in k or 'warmup' in k})"
