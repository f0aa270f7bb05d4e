"""Public multi-GPU path, end to end: `zest_amd.pull(repo, device="all")` of a synthetic model layout
served by an HBM seeder over BEP XET (loopback TCP), timed at N ranks.

Every Xet byte must come from the peer: the fake Hub publishes metadata only (`add_world(payload=
False)`), so a CDN xorb GET would 404 (counted).  N = 1 runs one rank with a one-rank process group;
N > 1 is a *rehearsal* on one GPU (ranks share cuda:0 over a gloo group, peer-mapped arenas through
HIP VMM where they map): its aggregate is not an xGMI number, but it runs every step of the multi-GPU
pull -- term shards, per-round agreement, autotuned exchange, receive-side hashing, Merkle checks.

Reports per rank: seconds, GB/s, bytes fetched (by source: peer / CDN / cache) vs received from
peer ranks, the exchange strategy and its autotune timings, and per-phase seconds (plan, map,
autotune, fetch, agree, exchange issue, verify).  Reference harness of the same shape:
test/local/p2p-docker-test.sh:112-218 (seeder + leecher, timed pull, p2p ratio).

    python tools/swarm_bench.py [--model llama-3.1-8b] [--ranks 1,2] [--out profiles/swarm_pull.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _rank(rank, world, port, repo, peer, env, q, threads, round_mb, exchange):
    import torch
    import torch.distributed as dist

    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    backend = "nccl" if world == 1 else "gloo"
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    try:
        import zest_amd
        from zest_amd.parallel import swarm_pull
        st: dict = {}
        dist.barrier()
        t0 = time.perf_counter()
        out = swarm_pull(repo, device="cuda:0", peers=[peer], dht=False, threads=threads, stats=st,
                         round_bytes=round_mb << 20, exchange=exchange)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        dist.barrier()
        n = sum(v.numel() * v.element_size() for v in out.values())
        del out, zest_amd
        q.put((rank, "ok", dict(st, wall_s=round(dt, 4), tensor_bytes=n)))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, "error", f"{type(e).__name__}: {e}\n{traceback.format_exc()[-3000:]}"))
    finally:
        dist.destroy_process_group()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3.1-8b")
    ap.add_argument("--ranks", default="1,2")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--round-mb", type=int, default=1024)
    ap.add_argument("--exchange", default="auto")
    ap.add_argument("--mode", default="random", choices=["random", "bf16"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch
    import torch.multiprocessing as mp

    from zest_amd import models, ops
    from zest_amd.seed import HbmSeedServer, HbmXorbArena
    from zest_amd.synthetic import SyntheticWorld
    from zest_amd.testing import FakeHub

    dev = torch.device("cuda:0")
    spec = models.get(a.model)
    t0 = time.time()
    world = SyntheticWorld(spec, seed=11, mode=a.mode, compression="bg4" if a.mode == "bf16" else "none")
    content = ops.padded_empty(world.arena_bytes, dev)
    world.generate_on_device(content)
    world.build_on_device(content)
    arena = HbmXorbArena(world, content)
    del content
    torch.cuda.empty_cache()
    srv = HbmSeedServer(arena)
    hub = FakeHub()
    hub.start()
    hub.add_world(world, exact=True, payload=False)
    total = world.model_bytes
    peer = f"127.0.0.1:{srv.port}"
    print(f"[setup] {spec.repo_id}: {total / 1e9:.2f} GB ({a.mode}, stored/raw "
          f"{float(world.chunk_clen.sum()) / float(world.chunk_len.sum()):.3f}), {world.n_chunks} chunks, "
          f"{world.n_xorbs} xorbs served from HBM on {peer} ({time.time() - t0:.1f}s)", flush=True)
    res = {"model": a.model, "repo": spec.repo_id, "bytes": total, "mode": a.mode,
           "source": "HBM seeder over BEP XET (loopback TCP); fake Hub metadata only (CDN xorb GETs 404)",
           "note": "N > 1 = ranks sharing one MI355X over gloo (rehearsal, not an xGMI number)", "runs": []}
    work = Path(tempfile.mkdtemp(prefix="zest-swarm-"))
    try:
        for n in [int(x) for x in a.ranks.split(",") if x]:
            env = hub.env(str(work / f"n{n}"))  # fresh caches per run: every byte comes from the seeder
            ctx = mp.get_context("spawn")
            q = ctx.Queue()
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            before = hub.counters.get("xorb_missing", 0) + hub.counters.get("xorb_get", 0)
            served0 = srv.stats()
            procs = [ctx.Process(target=_rank, args=(r, n, port, spec.repo_id, peer, env, q, a.threads, a.round_mb,
                                                     a.exchange)) for r in range(n)]
            t_run = time.perf_counter()
            for p in procs:
                p.start()
            out = sorted((q.get(timeout=1500) for _ in procs), key=lambda r: r[0])
            for p in procs:
                p.join(timeout=120)
            wall = time.perf_counter() - t_run
            errs = [r for r in out if r[1] != "ok"]
            if errs:
                print(f"[N={n}] failed: {errs}", flush=True)
                res["runs"].append({"ranks": n, "error": [e[2] for e in errs]})
                continue
            sts = [r[2] for r in out]
            pull_s = max(s["wall_s"] for s in sts)
            fetched = sum(s["fetched_bytes"] for s in sts)
            from_peer = sum(s["from_peer"] for s in sts)
            run = {"ranks": n, "pull_s": round(pull_s, 3), "aggregate_GBps": round(n * total / pull_s / 1e9, 3),
                   "per_rank_GBps": round(total / pull_s / 1e9, 3), "launch_wall_s": round(wall, 2),
                   "exchange": sts[0]["exchange"], "exchange_autotune_s": sts[0]["exchange_autotune_s"],
                   "network_bytes": fetched, "network_from_peer": from_peer,
                   "network_p2p_ratio": round(from_peer / fetched, 4) if fetched else 0.0,
                   "intra_node_p2p_ratio": round(sum(s["received_bytes"] for s in sts) / (n * total), 4),
                   "cdn_xorb_gets": hub.counters.get("xorb_missing", 0) + hub.counters.get("xorb_get", 0) - before,
                   "seeder_bytes_served": srv.stats().get("bytes_served", 0) - served0.get("bytes_served", 0),
                   "per_rank": [{k: s[k] for k in ("fetched_bytes", "received_bytes", "from_peer", "from_cdn",
                                                   "from_cache", "rounds", "items", "wall_s", "phases")} for s in sts]}
            res["runs"].append(run)
            print(f"[N={n}] pull(device='all'): {pull_s:.2f}s, {run['aggregate_GBps']:.2f} GB/s aggregate "
                  f"({run['per_rank_GBps']:.2f} per rank), exchange {run['exchange']}, network p2p ratio "
                  f"{run['network_p2p_ratio']}, intra-node {run['intra_node_p2p_ratio']}; phases rank0 "
                  f"{sts[0]['phases']}", flush=True)
        res["seeder"] = srv.stats()
        print(json.dumps(res), flush=True)
        if a.out:
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
        return 0
    finally:
        srv.stop()
        hub.stop()
        import shutil
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    raise SystemExit(main())
