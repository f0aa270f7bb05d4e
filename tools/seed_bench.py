#!/usr/bin/env python3
"""Seed-mode benchmark (BASELINE.json config 5): a synthetic model's xorbs live in HBM and are
served over BEP XET to concurrent loopback peers; reports chunks_served/s (CHUNK_RESPONSE messages,
the reference's unit, server.zig:196,208), GB/s, and the Xet chunks carried per second.

    python tools/seed_bench.py --model mixtral-8x7b --clients 16 --seconds 20

Each client holds one persistent connection and pipelines requests for whole xorbs (the unit a
puller asks for when a term spans a xorb) picked uniformly at random; every response is checked
for the requested chunk count on the client side (sizes) and a sample is hash-verified.
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from zest_amd import _core, models, ops  # noqa: E402
from zest_amd.seed import HbmSeedServer, HbmXorbArena  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mixtral-8x7b")
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--pipeline", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.time()
    world = SyntheticWorld(models.get(a.model), seed=a.seed)
    content = ops.padded_empty(world.arena_bytes, dev)
    world.generate_on_device(content)
    world.build_on_device(content)
    xa = HbmXorbArena(world, content)
    del content
    torch.cuda.empty_cache()
    srv = HbmSeedServer(xa)
    setup_s = time.time() - t0
    print(json.dumps({"setup_s": round(setup_s, 1), "model_bytes": world.model_bytes, "xorbs": len(xa.xorb_hex),
                      "hbm_xorb_bytes": xa.nbytes, "port": srv.port}), flush=True)

    # correctness sample: one xorb fetched and its chunk hashes checked on the host
    conn = _core.PeerConnection(f"127.0.0.1:{srv.port}", xa.xorb_hashes[0])
    data, off = conn.fetch(xa.xorb_hashes[0], 0, 0)
    info = _core.verify_xorb(data) if hasattr(_core, "verify_xorb") else None
    idx = _core.index_chunks(data)
    assert off == 0 and len(idx) == len(xa.xorb_ends[0]), "sample xorb mismatch"
    got = [_core.chunk_hash(data[e[0] + 8:e[0] + 8 + e[1]]) for e in idx[:16]]
    c0 = int(world.xorb_chunk0[0])
    want = [world.chunk_hashes[c0 + i].tobytes() for i in range(len(got))]
    assert got == want, "served chunk bytes do not hash to the published chunk hashes"
    del info

    stop = time.time() + a.seconds
    totals = {"bytes": 0, "reqs": 0, "chunks": 0, "failed": 0}
    lock = threading.Lock()
    n_x = len(xa.xorb_hex)
    nck = [len(e) for e in xa.xorb_ends]

    def client(k):
        rng = np.random.default_rng(1000 + k)
        c = _core.PeerConnection(f"127.0.0.1:{srv.port}", xa.xorb_hashes[0])
        while time.time() < stop:
            xs = rng.integers(0, n_x, a.pipeline)
            hs = [xa.xorb_hashes[x] for x in xs]
            b, failed = c.fetch_many_bytes(hs, [0] * len(xs), [nck[x] for x in xs])
            with lock:
                totals["bytes"] += b
                totals["reqs"] += len(xs)
                totals["chunks"] += sum(nck[x] for x in xs)
                totals["failed"] += failed

    t1 = time.time()
    st0 = srv.stats()
    ths = [threading.Thread(target=client, args=(k,)) for k in range(a.clients)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.time() - t1
    st1 = srv.stats()
    units = st1["chunk_units"] - st0["chunk_units"]
    responses = st1["chunks_served"] - st0["chunks_served"]
    # The reference's chunks_served counts CHUNK_RESPONSE messages (server.zig:196,208): that is
    # the headline unit here too.  Xet chunks inside those responses are reported separately.
    out = {"metric": "seed chunks_served/s (CHUNK_RESPONSEs) from HBM (loopback BEP XET peers)",
           "model": world.spec.repo_id, "clients": a.clients, "pipeline": a.pipeline, "seconds": round(dt, 2),
           "chunks_served_per_s": round(responses / dt, 1), "GBps": round(totals["bytes"] / dt / 1e9, 3),
           "xet_chunks_per_s": round(totals["chunks"] / dt, 1), "chunk_units_64KiB_per_s": round(units / dt, 1),
           "requests_per_s": round(totals["reqs"] / dt, 1), "failed": totals["failed"],
           # where the server's connection threads spent the window (seconds summed over connections):
           # queueing the HBM -> pinned copies, waiting for copied pieces, writing the sockets
           "server_split_s": {k: round(st1.get(k, 0.0) - st0.get(k, 0.0), 3) for k in ("lookup_s", "wait_s", "send_s")},
           "server": st1}
    print(json.dumps(out), flush=True)
    srv.stop()


if __name__ == "__main__":
    main()
