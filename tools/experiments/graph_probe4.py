"""Bisect the engine-step capture crash with the engine's own buffers and streams, re-issuing the
step's stream/event structure by hand: python tools/experiments/graph_probe4.py <flags>
flags: e = eager pass before capture (as capture_graph does), z = hashes.zero_() on the capture
stream, c = ws.chunks zero_ per round, r = the engine's lane streams (else fresh default-priority ones).
(Reproduces the copy-stream pipeline the engine used before round 2's per-lane copies.)"""
import faulthandler
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from zest_amd import ops  # noqa: E402
from zest_amd.engine import DevicePuller  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402

faulthandler.enable()
flags = sys.argv[1] if len(sys.argv) > 1 else ""
dev = torch.device("cuda:0")
H = ops.hip()
w = SyntheticWorld("llama-tiny", seed=10, mode="bf16", max_xorb_bytes=256 << 10)
arena = ops.padded_empty(w.arena_bytes, dev)
w.generate_on_device(arena)
w.build_on_device(arena)
p = DevicePuller(w, arena, 0, 1, round_bytes=256 << 10)
p.build_origin()
copy_s = torch.cuda.Stream(dev)
lanes = (p.lane_stream, p.side_stream) if "r" in flags else (torch.cuda.Stream(dev), torch.cuda.Stream(dev))


def body():
    main = torch.cuda.current_stream(dev)
    if "z" in flags:
        p.hashes.zero_()
    for ln in lanes:
        ln.wait_stream(main)
    copy_s.wait_stream(main)
    h2d_ev = [torch.cuda.Event() for _ in p.rounds]
    free_ev = [torch.cuda.Event() for _ in p.rounds]
    for k, rw in enumerate(p.rounds):
        s = k % p.slots
        comp, ws = lanes[k % 2], p.ws_lanes[k % 2]
        with torch.cuda.stream(copy_s):
            if k >= p.slots:
                copy_s.wait_event(free_ev[k - p.slots])
            if rw.span_len:
                H.memcpy_async(p.staging[s].data_ptr(), p.origin.ptr + rw.span_off, rw.span_len, copy_s.cuda_stream)
            h2d_ev[k].record(copy_s)
        with torch.cuda.stream(comp):
            comp.wait_event(h2d_ev[k])
            if "c" in flags and rw.term_b > rw.term_a:
                ws.chunks[: rw.n_chunks * ops.CHUNK_DTYPE.itemsize].zero_()
            if k + p.slots < p.n_rounds:
                free_ev[k].record(comp)
    for ln in lanes:
        main.wait_stream(ln)
    main.wait_stream(copy_s)


if "e" in flags:
    p.step()
    torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
print(f"[{flags}] captured", flush=True)
g.replay()
torch.cuda.synchronize()
print(f"[{flags}] replayed", flush=True)
