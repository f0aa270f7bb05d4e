#!/usr/bin/env python3
"""Time swarm_pull's plan requests (repo listing + every file's CAS reconstruction) against the
in-process fake hub holding Llama-3.1-70B-shaped metadata (no payload, no GPU): separates the hub's
and the HTTP client's cost from anything the bench process does.

    python tools/plan_probe.py [--model llama-3.1-70b] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from zest_amd import _core, models  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402
from zest_amd.testing import FakeHub  # noqa: E402


def fake_world(name: str) -> SyntheticWorld:
    """The model's files cut into 64 KiB chunks with random hashes (metadata only)."""
    w = SyntheticWorld(models.get(name), seed=0, mode="random")
    rng = np.random.default_rng(0)
    lens, owner = [], []
    for i, f in enumerate(w.xet_files):
        n, r = divmod(f.size, 65536)
        ln = np.full(n, 65536, np.int64)
        if r:
            ln = np.append(ln, r)
        lens.append(ln)
        owner.append(np.full(len(ln), i))
    w.chunk_len = np.concatenate(lens).astype(np.uint32)
    w.chunk_file = np.concatenate(owner).astype(np.int32)
    w.chunk_hashes = rng.integers(0, 256, (len(w.chunk_len), 32), dtype=np.uint8)
    w.chunk_off = np.concatenate([[0], np.cumsum(w.chunk_len.astype(np.uint64))[:-1]])
    w.chunk_clen = None
    w._plan_xorbs()
    w.file_hashes = rng.integers(0, 256, (len(w.xet_files), 32), dtype=np.uint8)
    return w


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3.1-70b")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    t = time.perf_counter()
    w = fake_world(a.model)
    hub = FakeHub()
    hub.xorb_url = "mem://probe"
    hub.start()
    hub.add_world(w, exact=True, payload=False)
    setup = time.perf_counter() - t
    for k, v in hub.env(tempfile.mkdtemp()).items():
        os.environ[k] = v
    f = _core.HostXetFetcher(w.spec.repo_id, p2p=False, dht=False)
    res = {"model": w.spec.repo_id, "files": len(w.xet_files), "terms": int(len(w.terms)), "setup_s": round(setup, 3)}
    for rep in range(a.reps):
        t = time.perf_counter()
        _, files = _core.list_repo_files(w.spec.repo_id, "main", "model")
        t_list = time.perf_counter() - t
        xet = [x for x in files if x["xet_hash"]]
        f.reset_reconstructions()
        t = time.perf_counter()
        with ThreadPoolExecutor(16) as ex:
            list(ex.map(lambda x: f.term_shapes(x["xet_hash"]), xet))
        t_rec = time.perf_counter() - t
        t = time.perf_counter()
        for x in xet:
            hub.reconstruction(x["xet_hash"])
        t_hub = time.perf_counter() - t
        res[f"rep{rep}"] = {"list_s": round(t_list, 4), "reconstructions_s": round(t_rec, 4),
                            "hub_compute_only_s": round(t_hub, 4)}
    print(json.dumps(res), flush=True)
    hub.stop()


if __name__ == "__main__":
    main()
