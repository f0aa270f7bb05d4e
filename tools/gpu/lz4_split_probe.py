"""Where the GPU LZ4/BG4 decoder's time goes (k_lz4_pair, producer parse || consumer execute).

    python tools/gpu/lz4_split_probe.py [--mib 256 1024] [--runs 5]

Builds N(0, 0.02) bf16 weights as BG4-LZ4 xorbs (the gpubench `lz4_decode_gpu_hostidx` data), takes
the chunk records from the host header walk, and times one fused decode + hash launch over:

  * all chunks (the real launch), checked byte-exact, with the dynamic chunk schedule (default) and
    the static one (ZG_PAIR_DYNAMIC=0), and without the parse's stream prefetch (ZG_PAIR_PREFETCH=0);
  * all chunks with ZG_PAIR_DEBUG=1 -- the consumer wave takes the records without executing them,
    so the launch times the parse alone (its size errors are expected and ignored); and with
    ZG_PAIR_DEBUG=2 -- parse and execute, but no BG4 ungroup and no fused hash;
  * only the largest quarter of the chunks, and only the smallest quarter: with one chunk per
    producer/consumer pair (a 256 MiB batch is ~4 k chunks for 4 k resident pairs) a launch lasts as
    long as its slowest chunk.

Prints one JSON line per size.  Diagnostics only; nothing here is on the pull path.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> int:
    import torch

    from zest_amd import _core, ops
    from zest_amd.gpubench import _bf16, _time, _xorb_runs

    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, nargs="+", default=[256, 1024])
    ap.add_argument("--runs", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    H = ops.hip()
    st = torch.cuda.current_stream(dev).cuda_stream
    for mib in a.mib:
        raw = _bf16(mib << 20)
        blob, terms, nck = _xorb_runs(raw, "bg4")
        src = ops.padded_empty(len(blob), dev)
        src.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
        dst = ops.padded_empty(len(raw), dev)
        hashes = torch.empty((nck, 32), dtype=torch.uint8, device=dev)
        ws = ops.IngestWorkspace(dev, len(terms), nck)
        pin = torch.frombuffer(bytearray(blob), dtype=torch.uint8).pin_memory()
        rec = np.zeros(nck, dtype=ops.CHUNK_DTYPE)
        th = np.ascontiguousarray(terms, dtype=ops.TERM_DTYPE)
        e = _core.index_runs(pin.data_ptr(), len(blob), th.ctypes.data, len(th), rec.ctypes.data, nck)
        if e:
            raise RuntimeError(f"host header walk failed ({e:#x})")
        sp, sb = ws.hash_scratch.get(nck, len(raw))

        def launch(sel: np.ndarray):
            r = np.ascontiguousarray(rec[sel])
            t = torch.from_numpy(r.view(np.uint8)).to(dev)

            def go():
                H.ingest_chunks(src.data_ptr(), len(blob), dst.data_ptr(), dst.numel(), t.data_ptr(), len(r), True,
                                ws.err.data_ptr(), hashes.data_ptr(), 0, 0, st, sp, sb)
            return go

        allc = np.arange(nck)
        comp = allc[rec["scheme"] != 0]
        order = comp[np.argsort(rec["ulen"][comp])]
        q = max(1, len(order) // 4)
        out = {"mib": mib, "chunks": int(nck), "compressed_chunks": int(len(comp)),
               "ulen_mean": float(rec["ulen"][comp].mean()), "ulen_max": int(rec["ulen"][comp].max())}
        ws.err.zero_()
        ns = _time(launch(allc), a.runs)
        torch.cuda.synchronize()
        ops.raise_on_error(ws.err)
        if dst[:len(raw)].cpu().numpy().tobytes() != raw:
            raise RuntimeError("decoded bytes differ from the input")
        out["all_ms"] = round(ns / 1e6, 3)
        out["all_GBps"] = round(len(raw) / ns, 2)
        os.environ["ZG_PAIR_DYNAMIC"] = "0"  # the static chunk schedule (block b: chunks b, b + grid, ...)
        try:
            dst.zero_()
            ns_s = _time(launch(allc), a.runs)
            torch.cuda.synchronize()
            ops.raise_on_error(ws.err)
            if dst[:len(raw)].cpu().numpy().tobytes() != raw:
                raise RuntimeError("decoded bytes differ from the input (static schedule)")
        finally:
            os.environ.pop("ZG_PAIR_DYNAMIC", None)
        os.environ["ZG_PAIR_PREFETCH"] = "0"  # no L2 prefetch of the compressed stream ahead of the parse
        try:
            dst.zero_()
            ns_p = _time(launch(allc), a.runs)
            torch.cuda.synchronize()
            ops.raise_on_error(ws.err)
            if dst[:len(raw)].cpu().numpy().tobytes() != raw:
                raise RuntimeError("decoded bytes differ from the input (no prefetch)")
        finally:
            os.environ.pop("ZG_PAIR_PREFETCH", None)
        out["no_prefetch_ms"] = round(ns_p / 1e6, 3)
        out["no_prefetch_GBps"] = round(len(raw) / ns_p, 2)
        out["static_ms"] = round(ns_s / 1e6, 3)
        out["static_GBps"] = round(len(raw) / ns_s, 2)
        os.environ["ZG_FUSED_HASH"] = "0"  # decode only, then the place/hash pass hashes every chunk
        try:
            dst.zero_()
            ns_u = _time(launch(allc), a.runs)
            torch.cuda.synchronize()
            ops.raise_on_error(ws.err)
            if dst[:len(raw)].cpu().numpy().tobytes() != raw:
                raise RuntimeError("decoded bytes differ from the input (unfused hash)")
        finally:
            os.environ.pop("ZG_FUSED_HASH", None)
        out["unfused_hash_ms"] = round(ns_u / 1e6, 3)
        out["unfused_hash_GBps"] = round(len(raw) / ns_u, 2)
        out["largest_quarter_ms"] = round(_time(launch(order[-q:]), a.runs) / 1e6, 3)
        out["smallest_quarter_ms"] = round(_time(launch(order[:q]), a.runs) / 1e6, 3)
        os.environ["ZG_PAIR_DEBUG"] = "1"
        try:
            out["parse_only_ms"] = round(_time(launch(allc), a.runs) / 1e6, 3)
            os.environ["ZG_PAIR_DEBUG"] = "2"  # parse + execute, no ungroup / hash
            out["no_ungroup_hash_ms"] = round(_time(launch(allc), a.runs) / 1e6, 3)
        finally:
            os.environ.pop("ZG_PAIR_DEBUG", None)
            torch.cuda.synchronize()
            ws.err.zero_()
        print(json.dumps(out), flush=True)
        del src, dst, hashes, ws, pin
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
