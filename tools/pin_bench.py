#!/usr/bin/env python3
"""Concurrent pinning cost: N processes each pin G GB of host memory at the same moment, the way
the N ranks of an 8-GPU bench pin their origin shares (1/N of a 141 GB Llama-3.1-70B each) during
setup.  Each child allocates through the same path as OriginStore (`ops.hip().host_malloc`:
THP-advised mmap, parallel fault-in, hipHostRegister) and reports how long pinning and freeing took.

    python tools/pin_bench.py --procs 8 --gb 17.6 [--out f.json]

The parent never touches the GPU (children start as fresh processes); children start pinning at a
common wall-clock instant after their imports.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child(gb: float, start_at: float) -> None:
    sys.path.insert(0, str(ROOT))
    from zest_amd import ops
    H = ops.hip()
    n = int(gb * 1e9)
    time.sleep(max(0.0, start_at - time.time()))
    t0 = time.time()
    ptr = H.host_malloc(n)
    t1 = time.time()
    H.host_free(ptr)
    t2 = time.time()
    print(json.dumps({"pid": os.getpid(), "late_s": round(t0 - start_at, 3), "pin_s": round(t1 - t0, 3),
                      "free_s": round(t2 - t1, 3), "start": t0, "end_pin": t1}), flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--gb", type=float, default=17.6)
    ap.add_argument("--delay", type=float, default=45.0, help="seconds for the children's imports")
    ap.add_argument("--out", default=None)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--start-at", type=float, default=0.0)
    a = ap.parse_args()
    if a.child:
        child(a.gb, a.start_at)
        return 0
    start_at = time.time() + a.delay
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", "--gb", str(a.gb),
                               "--start-at", repr(start_at)], stdout=subprocess.PIPE, text=True, env=env)
             for _ in range(a.procs)]
    rows, rc = [], 0
    for p in procs:
        out, _ = p.communicate()
        rc |= p.returncode
        rows += [json.loads(line) for line in out.splitlines() if line.startswith("{")]
    if rc or len(rows) != a.procs:
        print(f"pin_bench: {len(rows)} of {a.procs} children reported (rc {rc})", file=sys.stderr)
        return 1
    span = max(r["end_pin"] for r in rows) - min(r["start"] for r in rows)
    res = {"procs": a.procs, "gb_each": a.gb, "total_gb": round(a.procs * a.gb, 1),
           "pin_s_max": max(r["pin_s"] for r in rows), "pin_s_min": min(r["pin_s"] for r in rows),
           "all_pinned_after_s": round(span, 3), "aggregate_GBps": round(a.procs * a.gb / span, 2),
           "free_s_max": max(r["free_s"] for r in rows), "late_s_max": max(r["late_s"] for r in rows),
           "per_proc": [{k: r[k] for k in ("pin_s", "free_s", "late_s")} for r in rows]}
    print(json.dumps(res), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
