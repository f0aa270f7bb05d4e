"""Minimal HIP-graph capture shapes of the engine step (no engine code):
python tools/experiments/graph_probe3.py <variant>  A full shape, B no memsets on the lanes, C one lane,
D copies issued on the lanes (no copy stream), E copy stream only (no lanes), P = A on
high-priority streams (as the engine creates them), X = A + the copy stream waiting on lane events."""
import faulthandler
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from zest_amd import ops  # noqa: E402

faulthandler.enable()
v = sys.argv[1]
dev = torch.device("cuda:0")
H = ops.hip()
R, n = 17, 1 << 20
host = H.host_malloc(R * n)
staging = [ops.padded_empty(n, dev) for _ in range(3)]
small = [torch.empty(4096, dtype=torch.uint8, device=dev) for _ in range(2)]
pri = int(torch.cuda.Stream.priority_range()[1]) if v == "P" else 0
copy_s = torch.cuda.Stream(dev, priority=pri)
lanes = [torch.cuda.Stream(dev, priority=pri), torch.cuda.Stream(dev, priority=pri)] if v != "C" else [torch.cuda.Stream(dev)]
g = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    main = torch.cuda.current_stream()
    ev_h2d = [torch.cuda.Event() for _ in range(R)]
    ev_free = [torch.cuda.Event() for _ in range(R)]
    if v != "E":
        for ln in lanes:
            ln.wait_stream(main)
    if v != "D":
        copy_s.wait_stream(main)
    for k in range(R):
        ln = lanes[k % len(lanes)]
        if v == "D":
            H.memcpy_async(staging[k % 3].data_ptr(), host + k * n, n, ln.cuda_stream)
        else:
            if v == "X" and k >= 3:  # the copy stream waits for a lane (staging slot reuse)
                copy_s.wait_event(ev_free[k - 3])
            H.memcpy_async(staging[k % 3].data_ptr(), host + k * n, n, copy_s.cuda_stream)
            ev_h2d[k].record(copy_s)
            if v != "E":
                ln.wait_event(ev_h2d[k])
        if v not in ("B", "E"):
            with torch.cuda.stream(ln):
                small[k % 2].zero_()
        if v == "X" and k + 3 < R:
            ev_free[k].record(ln)
    if v != "E":
        for ln in lanes:
            main.wait_stream(ln)
    if v != "D":
        main.wait_stream(copy_s)
print(f"{v}: captured", flush=True)
g.replay()
torch.cuda.synchronize()
print(f"{v}: replayed", flush=True)
