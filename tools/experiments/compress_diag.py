"""Per-input GPU vs host LZ4/BG4 compressed sizes (diagnostic for the K7b kernel)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
import torch
from zest_amd import _core, ops
rng = np.random.default_rng(5)
w = (rng.standard_normal(300_000).astype(np.float32) * 0.02)
bf16 = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
parts = {"bf16_64k": bf16[:65536], "bf16_128k": bf16[65536:65536 + 131072],
         "lowent": rng.integers(0, 8, 70_000, dtype=np.uint8).tobytes(), "zeros": bytes(40_000),
         "text": (b"the quick brown fox jumps over the lazy dog " * 2000)[:60000]}
blob = b"".join(parts.values())
lens = np.array([len(p) for p in parts.values()], dtype=np.uint32)
offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
buf = ops.padded_empty(len(blob), torch.device("cuda:0"))
buf.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
for bg4 in (True, False):
    _, flen = ops.compress_chunks(buf, offs, lens, bg4=bg4)
    for (name, p), g in zip(parts.items(), flen):
        h = len(_core.compress_chunk(p, "bg4" if bg4 else "lz4")[1])
        print(f"bg4={bg4} {name:10s} n={len(p):7d} gpu={int(g):7d} host={h:7d}")
