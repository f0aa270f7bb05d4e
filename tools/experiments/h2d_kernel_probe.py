#!/usr/bin/env python3
"""PCIe H2D probe, copy engines vs. a kernel reading pinned host memory (zero-copy, K8 gather
kernel pointed at host pages) vs. both at once on separate streams.  4 GiB per measurement."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from zest_amd import ops  # noqa: E402

H = ops.hip()
n = 4 << 30
host = H.host_malloc(n)
torch.cuda.synchronize()
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def kernel_copy(off, nb, st, segs=16):
    part = nb // segs
    src = [host + off + i * part for i in range(segs)]
    dst = [dev.data_ptr() + off + i * part for i in range(segs)]
    H.peer_gather(src, dst, [part] * segs, st.cuda_stream)


def run(name, dma_frac):
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        nd = int(n * dma_frac) & ~((1 << 20) - 1)
        s1.wait_event(e0)
        s2.wait_event(e0)
        if nd:
            H.memcpy_async(dev.data_ptr(), host, nd, s1.cuda_stream)
        if n - nd:
            kernel_copy(nd, n - nd, s2)
        torch.cuda.current_stream().wait_stream(s1)
        torch.cuda.current_stream().wait_stream(s2)
        e1.record()
        torch.cuda.synchronize()
        best = max(best, n / e0.elapsed_time(e1) / 1e6)
    print(json.dumps({"case": name, "dma_fraction": dma_frac, "GBps": round(best, 2)}), flush=True)


# correctness of the kernel path on host pages
hv = torch.from_numpy(__import__("numpy").frombuffer(
    (__import__("ctypes").c_uint8 * (1 << 20)).from_address(host), dtype="uint8"))
hv.copy_(torch.randint(0, 256, (1 << 20,), dtype=torch.uint8))
kernel_copy(0, 1 << 20, s2, segs=4)
torch.cuda.synchronize()
assert torch.equal(dev[: 1 << 20].cpu(), hv), "kernel H2D copy mismatch"
for name, f in (("dma", 1.0), ("kernel", 0.0), ("both_50", 0.5), ("both_75", 0.75), ("both_90", 0.9)):
    run(name, f)
H.host_free(host)
