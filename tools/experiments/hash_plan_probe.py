"""Probe: leaf-flat K1 kernels with a device sync between launches (kernel-trace durations without
back-to-back queueing effects).  python tools/experiments/hash_plan_probe.py [n_chunks] [chunk_bytes]"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from zest_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
cs = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
dev = torch.device("cuda:0")
H = ops.hip()
arena = ops.padded_empty(n * cs, dev)
ops.fill_synthetic(arena, 0, 0, 0)
offs = torch.from_numpy((np.arange(n, dtype=np.int64) * cs)).to(dev)
lens = torch.full((n,), cs, dtype=torch.int32, device=dev)
out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
hs = ops.HashScratch(dev)
sp, sb = hs.get(n, n * cs)
st = torch.cuda.current_stream().cuda_stream
for _ in range(4):
    torch.cuda.synchronize()
    H.hash_ranges(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), n, out.data_ptr(), 0, st, sp, sb)
    torch.cuda.synchronize()
print("ok", out[0, :4].tolist())
