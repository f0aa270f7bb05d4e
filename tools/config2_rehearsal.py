#!/usr/bin/env python3
"""BASELINE config 2 on the PUBLIC path: "Llama-3.1-8B pull, 2-GPU intra-node swarm (1 seeder + 1
leecher)", run as zest_amd.pull(repo, device="all") = parallel.swarm_pull.

Rank 0's xorb cache already holds the model (an earlier pull; here written from the synthetic
world's serialized runs), rank 1 starts cold.  The possession have-map (swarm_pull.gather_possession)
makes rank 0 the node's seeder: it owns every term, reads it from its cache through the normal
cache -> P2P -> CDN waterfall, decodes + hashes it on its GPU, and the exchange replicates it to
rank 1, which verifies everything itself.  The CDN is a mem:// origin with nothing registered: a
rank that tried it would fail, so a passing run proves no byte came from the network.

One-GPU boxes: both ranks share cuda:0 over gloo (ZEST_BENCH_BACKEND semantics): the exchange is the
peer-mapped HIP VMM path (ipc / xgmi kernel), not RCCL over xGMI.  With distinct GPUs per rank the
default group is RCCL.

    python tools/config2_rehearsal.py [--model llama-3.1-8b] [--mode bf16] [--ranks 2] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3.1-8b")
    ap.add_argument("--mode", default="bf16", choices=["bf16", "random"])
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--warm", default="0", help="comma list of ranks whose cache holds the model")
    ap.add_argument("--exchange", default="auto")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--steps", type=int, default=2, help="timed pulls (after one untimed warm-up pull)")
    ap.add_argument("--root", default=None, help="scratch directory (caches); default: a temp dir")
    ap.add_argument("--out", default=None)
    return ap.parse_args(argv)


def rank_main(a) -> None:
    import numpy as np
    import torch
    import torch.distributed as dist

    from zest_amd import _core, models, ops
    from zest_amd.engine import DevicePuller, release_pinned_pool
    from zest_amd.parallel.swarm_pull import swarm_pull
    from zest_amd.synthetic import SyntheticWorld
    from zest_amd.testing import FakeHub

    rank, world_size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    cuda = a.device == "cuda"
    if cuda:
        n_dev = max(1, torch.cuda.device_count())
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % n_dev)
        torch.cuda.set_device(device)
        backend = "nccl" if n_dev >= world_size and os.environ.get("ZEST_BENCH_BACKEND") != "gloo" else "gloo"
    else:
        device, backend = torch.device("cpu"), "gloo"
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group("gloo")
    root = Path(a.root)
    warm = {int(x) for x in a.warm.split(",") if x != ""}
    spec = models.get(a.model)
    t0 = time.time()
    comp = "bg4" if (a.mode == "bf16" and cuda) else "none"
    world = SyntheticWorld(spec, seed=11, mode=a.mode, compression=comp)
    if cuda:
        arena = ops.padded_empty(world.arena_bytes, device)
        world.generate_on_device(arena)
        world.build_on_device(arena)
        torch.cuda.synchronize()
    else:
        contents = world.build_on_host()
        arena = torch.zeros(world.arena_bytes + 4096, dtype=torch.uint8)[: world.arena_bytes]
    cache = root / f"cache{rank}"
    os.environ["ZEST_CACHE_DIR"] = str(cache)
    if rank in warm:  # this rank pulled the model before: its xorb cache holds every term's run
        p = DevicePuller(world, arena, 0, 1, round_bytes=1 << 30)
        if cuda:
            p.build_origin()
            torch.cuda.synchronize()
        else:
            p.build_origin_host(contents)
        T = world.terms
        n = len(T)
        _core.cache_put_runs([world.xorb_hash_hex(int(T["xorb"][t])) for t in range(n)],
                             [int(T["local0"][t]) for t in range(n)],
                             [p.origin.ptr + int(p.term_origin_off[t]) for t in range(n)],
                             [int(T["ser_len"][t]) for t in range(n)], 16)
        p.close()
        release_pinned_pool()
    del arena
    if cuda:
        torch.cuda.empty_cache()
    hub = FakeHub()
    hub.xorb_url = "mem://nothing-registered"  # any CDN fetch fails: every byte must come from a rank
    hub.start()
    hub.add_world(world, exact=True, payload=False)
    env = hub.env(str(root / f"home{rank}"))
    env["ZEST_CACHE_DIR"] = str(cache)
    os.environ.update(env)
    setup_s = time.time() - t0
    times, st = [], {}
    for i in range(1 + a.steps):
        st = {}
        dist.barrier()
        if cuda:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        out = swarm_pull(world.spec.repo_id, device=device if cuda else None, p2p=False, dht=False, stats=st,
                         exchange=a.exchange, reuse_pipeline=True)
        if cuda:
            torch.cuda.synchronize()
        dist.barrier()
        if i:
            times.append(time.perf_counter() - t1)
        n_tensors = len(out)
        del out
    mine = {"rank": rank, "device": str(device), "from_cache": st["from_cache"], "from_cdn": st["from_cdn"],
            "from_peer": st["from_peer"], "fetched_bytes": st["fetched_bytes"], "received_bytes": st["received_bytes"],
            "exchange": st["exchange"], "peer_mapped": st["peer_mapped"], "possession": st["possession"],
            "phases": st["phases"], "pull_s": [round(x, 4) for x in times], "tensors": n_tensors,
            "autotune_s": st.get("exchange_autotune_s")}
    every = [None] * world_size
    dist.all_gather_object(every, mine)
    if rank == 0:
        total = st["total_bytes"]
        step = max(max(r["pull_s"]) for r in every)
        res = {"config": "BASELINE config 2: 1 seeder + leechers, public swarm_pull path",
               "model": spec.repo_id, "data_mode": a.mode, "model_bytes": total, "ranks": world_size,
               "backend": backend, "warm_ranks": sorted(warm),
               "aggregate_GBps": round(world_size * total / step / 1e9, 3),
               "leecher_receive_GBps": round(total / step / 1e9, 3),
               "cdn_bytes": sum(r["from_cdn"] for r in every), "setup_s": round(setup_s, 2),
               "verify": "merkle file hashes of every file on every rank", "per_rank": every}
        print(json.dumps(res), flush=True)
        if a.out:
            Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
    from zest_amd.parallel.swarm_pull import release_pipelines
    release_pipelines()
    hub.stop()
    dist.barrier()
    dist.destroy_process_group()
    del np


def main(argv=None) -> int:
    a = parse(argv)
    if "WORLD_SIZE" in os.environ:
        rank_main(a)
        return 0
    root = a.root or tempfile.mkdtemp(prefix="zest-config2-")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    argv = sys.argv[1:] if argv is None else list(argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv,
           "--root", root]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    try:
        return subprocess.call(cmd, env=env)
    finally:
        if not a.root:
            shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    raise SystemExit(main())
