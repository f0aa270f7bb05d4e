#!/usr/bin/env python3
"""Where does a released peer-mapped VMM arena's device memory go?  

Two ranks share the one GPU (gloo).  Each iteration every rank allocates a VMM arena, optionally
exports / maps it into the peer (the real zest_amd.parallel.exchange.map_peer_arenas path), then
releases everything and waits for the driver's reclaim.  Device free memory is recorded after every
step, with the process's open fd count, for these modes (--modes, comma list):

  alloc     vmm_alloc + release only (no export)                      -> baseline
  export    + export every chunk as a dmabuf fd, close the fds          -> does an export pin memory?
  map       + the peer imports and maps the chunks (map_peer_arenas)    -> the swarm pull's path
  map_rev   like map, but the owners release before the importers
  map_fresh like map, the importer moving every received fd to a never-used fd number first

Usage: python tools/vmm_leak_probe.py [--gb 4] [--iters 3] [--modes alloc,export,map,map_rev]
Prints one JSON line per rank and mode.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _fds() -> int:
    try:
        return len(os.listdir("/proc/self/fd"))
    except OSError:
        return -1


def _free(torch, dev) -> float:
    return torch.cuda.mem_get_info(dev)[0] / 1e9


def _settle(torch, dev, quiet=0.5, limit=20.0) -> float:
    """Free device GB once it stopped growing (the driver reclaims freed memory asynchronously)."""
    t0 = time.time()
    last, since = _free(torch, dev), time.time()
    while time.time() - t0 < limit:
        time.sleep(0.05)
        f = _free(torch, dev)
        if f > last + 1e-3:
            last, since = f, time.time()
        elif time.time() - since >= quiet:
            break
    return last


def worker(rank, world, port, gb, iters, modes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZEST_IPC_DEBUG="1")
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zest_amd import ops
    from zest_amd.parallel.exchange import map_peer_arenas
    H = ops.hip()
    out = []
    try:
        for mode in modes:
            rec = {"rank": rank, "mode": mode, "steps": []}
            dist.barrier()
            base = _settle(torch, dev)
            rec["base_GB"] = round(base, 2)
            for it in range(iters):
                arena = ops.vmm_empty(int(gb * (1 << 30)), dev)
                torch.cuda.synchronize()
                a_free = _free(torch, dev)
                mapped = None
                if mode == "export":
                    for fd in ops.vmm_mapping(arena).export_fds():
                        os.close(fd)
                elif mode in ("map", "map_rev", "map_fresh"):
                    # (mapped while fresh, as the swarm pull and the bench do)
                    os.environ["ZEST_VMM_FRESH_FDS"] = "1" if mode == "map_fresh" else "0"
                    mapped = map_peer_arenas(arena, rank, world)
                mapped_ok = mapped is not None or mode in ("alloc", "export")
                arena.fill_(rank + 1)
                reads_ok = None
                if mapped is not None:  # the peer's bytes read back through the mapping
                    torch.cuda.synchronize()
                    dist.barrier()
                    peer = mapped.peers[1 - rank]
                    reads_ok = int(peer[:16].cpu()[0]) == 2 - rank
                    del peer
                torch.cuda.synchronize()
                dist.barrier()
                m_free = _free(torch, dev)
                fds_mapped = _fds()
                peers = mapped.peers if mapped is not None else None
                mapped = None  # (PeerArenas also references the own arena)
                if mode == "map_rev":  # owners first: drop the own arena, keep the peer's mapping
                    del arena
                    gc.collect()
                    torch.cuda.synchronize()
                    dist.barrier()
                    peers = None
                else:  # importers first
                    peers = None
                    gc.collect()
                    torch.cuda.synchronize()
                    dist.barrier()
                    del arena
                gc.collect()
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
                dist.barrier()
                f = _settle(torch, dev)
                own, imp = H.vmm_live()
                rec["steps"].append({"iter": it, "mapped": mapped_ok, "reads_ok": reads_ok,
                                     "after_alloc_GB": round(a_free, 2), "after_map_GB": round(m_free, 2),
                                     "after_release_GB": round(f, 2), "leaked_GB": round(base - f, 2),
                                     "fds_mapped": fds_mapped, "fds_after": _fds(),
                                     "vmm_live_own": own, "vmm_live_imported": imp})
                dist.barrier()
            out.append(rec)
            print(json.dumps(rec), flush=True)
    finally:
        q.put(out)
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--modes", default="alloc,export,map,map_rev,map_fresh")
    a = ap.parse_args()
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    modes = [m for m in a.modes.split(",") if m]
    ps = [ctx.Process(target=worker, args=(r, 2, port, a.gb, a.iters, modes, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    worst = max((s["leaked_GB"] for r in res for rec in r for s in rec["steps"]), default=0.0)
    print(json.dumps({"summary": {rec["mode"]: [(s["leaked_GB"], s["mapped"], s["reads_ok"]) for s in rec["steps"]]
                                  for r in res for rec in r if rec["rank"] == 0}, "worst_leak_GB": worst}), flush=True)


if __name__ == "__main__":
    main()
