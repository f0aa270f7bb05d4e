"""Probe: which part of a HIP-graph capture of the engine step crashes.  Stages run in order in one
process and print as they complete: (1) memcpy H2D from pinned host memory, (2) + our kernels,
(3) + a second stream joined by events, (4) the DevicePuller step on a tiny world."""
import faulthandler
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from zest_amd import ops  # noqa: E402

faulthandler.enable()
dev = torch.device("cuda:0")
H = ops.hip()
n = 1 << 20
host = torch.empty(n, dtype=torch.uint8).pin_memory()
host.copy_(torch.randint(0, 256, (n,), dtype=torch.uint8))
d = ops.padded_empty(n, dev)


def stage(name, body):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        body()
    print(f"{name}: captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"{name}: replayed", flush=True)
    return g


stage("1 torch copy_ H2D", lambda: d[:n].copy_(host, non_blocking=True))
stage("1b hipMemcpyAsync H2D", lambda: H.memcpy_async(d.data_ptr(), host.data_ptr(), n,
                                                       torch.cuda.current_stream().cuda_stream))
offs = torch.tensor([0, 4096], dtype=torch.int64, device=dev)
lens = torch.tensor([4096, 8192], dtype=torch.int32, device=dev)
out = torch.empty((2, 32), dtype=torch.uint8, device=dev)
stage("2 hash_ranges (wave kernel)", lambda: H.hash_ranges(d.data_ptr(), offs.data_ptr(), lens.data_ptr(), 2,
                                                            out.data_ptr(), 0, torch.cuda.current_stream().cuda_stream))
hs = ops.HashScratch(dev)
sp, sb = hs.get(2, 12288)
stage("2b hash_ranges (flat)", lambda: H.hash_ranges(d.data_ptr(), offs.data_ptr(), lens.data_ptr(), 2,
                                                      out.data_ptr(), 0, torch.cuda.current_stream().cuda_stream, sp, sb))
side = torch.cuda.Stream(dev)
ev = torch.cuda.Event()


def two_streams():
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        H.memcpy_async(d.data_ptr(), host.data_ptr(), n, side.cuda_stream)
        ev.record(side)
    main.wait_event(ev)
    H.hash_ranges(d.data_ptr(), offs.data_ptr(), lens.data_ptr(), 2, out.data_ptr(), 0, main.cuda_stream, sp, sb)


stage("3 two streams + events", two_streams)
from zest_amd.engine import DevicePuller  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402

w = SyntheticWorld("llama-tiny", seed=10, mode="bf16", max_xorb_bytes=256 << 10)
arena = ops.padded_empty(w.arena_bytes, dev)
w.generate_on_device(arena)
w.build_on_device(arena)
p = DevicePuller(w, arena, 0, 1, round_bytes=256 << 10)
p.build_origin()
print("4 puller ready, rounds", p.n_rounds, flush=True)
print("4 capture:", p.capture_graph(), flush=True)
p.step()
torch.cuda.synchronize()
p.check()
print("4 replay ok", flush=True)
