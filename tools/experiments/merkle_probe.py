"""Probe: K2 Merkle stages on 8 x 80k leaves (the gpubench merkle_gpu row), synced launches."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from zest_amd import ops  # noqa: E402

nl = 80_000
lh = torch.randint(0, 256, (nl * 8, 32), dtype=torch.uint8, device="cuda:0")
sz = torch.randint(8192, 131072, (nl * 8,), dtype=torch.int64, device="cuda:0")
jobs = [(i * nl, nl) for i in range(8)]
for _ in range(4):
    torch.cuda.synchronize()
    ops.merkle_roots(lh, sz, jobs)
    torch.cuda.synchronize()
print("ok")
