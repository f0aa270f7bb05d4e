"""Bisect the DevicePuller HIP-graph capture crash: python tools/experiments/graph_probe2.py <level>
level 0: H2D copies + events + torch memsets only (engine kernels stubbed out), 1: + index_terms,
2: + place_chunks, 3: + hash_chunks, 4: + merkle/compare (the full step)."""
import faulthandler
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from zest_amd import ops  # noqa: E402
from zest_amd.engine import DevicePuller  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402

faulthandler.enable()
level = int(sys.argv[1])
H = ops.hip()
names = ["index_terms", "place_chunks", "hash_chunks", "merkle", "compare_hashes"]
keep = {0: 0, 1: 1, 2: 2, 3: 3, 4: 5}[level]
for nm in names[keep:]:
    setattr(H, nm, lambda *a, **k: None)
dev = torch.device("cuda:0")
w = SyntheticWorld("llama-tiny", seed=10, mode="bf16", max_xorb_bytes=256 << 10)
arena = ops.padded_empty(w.arena_bytes, dev)
w.generate_on_device(arena)
w.build_on_device(arena)
p = DevicePuller(w, arena, 0, 1, round_bytes=256 << 10)
p.build_origin()
print(f"level {level}: stubbed {names[keep:]}; rounds {p.n_rounds}", flush=True)
print(f"level {level}: capture {p.capture_graph()}", flush=True)
p.step()
torch.cuda.synchronize()
print(f"level {level}: replay ok", flush=True)
