#!/usr/bin/env python3
"""PCIe H2D ceiling probe: pinned host -> HBM, one 4 GiB transfer split over 1/2/4 streams."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from zest_amd import ops  # noqa: E402

H = ops.hip()
n = 4 << 30
host = H.host_malloc(n)
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
for streams in (1, 2, 4):
    ss = [torch.cuda.Stream() for _ in range(streams)]
    part = n // streams
    for rep in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i, s in enumerate(ss):
            s.wait_event(e0)
            H.memcpy_async(dev.data_ptr() + i * part, host + i * part, part, s.cuda_stream)
        for s in ss:
            e1.wait_stream(s) if hasattr(e1, "wait_stream") else None
            torch.cuda.current_stream().wait_stream(s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
    print(json.dumps({"streams": streams, "GBps": round(n / ms / 1e6, 2)}), flush=True)
H.host_free(host)
