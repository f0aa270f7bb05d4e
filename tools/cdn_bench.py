#!/usr/bin/env python3
"""BASELINE config 0: `zest pull <gpt2> --no-p2p` on the CPU (CDN-only plumbing: Xet listing,
reconstruction, ranged xorb fetches, LZ4/BG4 decode and BLAKE3/Merkle verification on the host).

No network exists, so an in-process fake Hub/CAS on loopback serves a synthetic repository with the
real GPT-2 tensor shapes (bf16-like weights, so the hub's `auto` policy stores BG4-LZ4 chunks the
way Xet does for real checkpoints).  Prints one JSON line; a second pull shows the local-cache path
(the reference's "< 1 s re-download" target, DESIGN.md:572).

    python tools/cdn_bench.py [--model gpt2] [--runs 3]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    from e2e_util import ZEST, Node
    from zest_amd.synthetic import SyntheticWorld
    from zest_amd.testing import FakeHub

    world = SyntheticWorld(a.model, seed=1, mode="bf16")
    hub = FakeHub(policy="auto")
    hub.start()
    tmp = Path(tempfile.mkdtemp(prefix="zest_cdn_bench_"))
    try:
        t0 = time.time()
        commit = hub.add_world(world)
        publish_s = time.time() - t0
        total = sum(f.size for f in world.files)
        cold, warm = [], []
        for i in range(a.runs):
            n = Node(hub, tmp, f"run{i}")
            t0 = time.perf_counter()
            r = n.run("pull", world.spec.repo_id, "--no-p2p", "--no-dht", timeout=1200)
            cold.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            n.run("pull", world.spec.repo_id, "--no-p2p", "--no-dht", timeout=1200)
            warm.append(time.perf_counter() - t0)
            snap = n.snapshot(world.spec.repo_id, commit)
            assert all((snap / f.path).stat().st_size == f.size for f in world.files)
            shutil.rmtree(n.root)
        stored = sum(len(x.data) for x in hub.xorbs)
        best = min(cold)
        print(json.dumps({"config": "BASELINE configs[0]: pull --no-p2p on CPU", "model": world.spec.repo_id,
                          "bytes": total, "xorb_bytes_stored": stored, "compression_ratio": round(stored / total, 4),
                          "cold_pull_s": [round(x, 3) for x in cold], "cold_GBps": round(total / best / 1e9, 3),
                          "cached_repull_s": [round(x, 3) for x in warm], "publish_s": round(publish_s, 1),
                          "cpus": os.cpu_count(), "cdn": "fake Hub/CAS on 127.0.0.1 (no network)",
                          "last_stdout_tail": r.stdout.strip().splitlines()[-6:]}))
    finally:
        hub.stop()
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
