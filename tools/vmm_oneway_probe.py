#!/usr/bin/env python3
"""Who keeps a released, peer-imported VMM allocation alive?  (follow-up of tools/vmm_leak_probe.py)

Rank 0 allocates a VMM arena and exports its chunks (dmabuf fds over an abstract Unix socket); rank 1
alone imports and maps them (one direction), checks the bytes, then releases its mapping; rank 0 then
releases its arena; finally rank 1's PROCESS exits while rank 0 keeps measuring.  Device free memory
(both ranks share the GPU) after each step says which process's runtime still holds the memory:

  leak after both released, gone after the importer exited -> the importer's runtime holds it
  leak still there after the importer exited                -> the exporter's runtime holds it

Usage: python tools/vmm_oneway_probe.py [--gb 4]; prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _settle(torch, dev, quiet=0.5, limit=15.0) -> float:
    t0 = time.time()
    last, since = torch.cuda.mem_get_info(dev)[0], time.time()
    while time.time() - t0 < limit:
        time.sleep(0.05)
        f = torch.cuda.mem_get_info(dev)[0]
        if f > last + (1 << 20):
            last, since = f, time.time()
        elif time.time() - since >= quiet:
            break
    return last / 1e9


def worker(rank, port, gb, q, ev):
    import torch
    from torch.utils.dlpack import from_dlpack

    from zest_amd import ops
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    H = ops.hip()
    name = f"\0zest-oneway-{port}"
    n = int(gb * (1 << 30))
    out = {}
    if rank == 0:
        base = _settle(torch, dev)
        arena = ops.vmm_empty(n, dev)
        arena.fill_(7)
        torch.cuda.synchronize()
        vm = ops.vmm_mapping(arena)
        fds = vm.export_fds()
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        srv.bind(name)
        srv.listen(1)
        ev["listening"].set()
        conn, _ = srv.accept()
        for i in range(0, len(fds), 200):
            socket.send_fds(conn, [b"z"], fds[i:i + 200])
        conn.recv(1)  # the importer holds its own references now
        for fd in fds:
            os.close(fd)
        out["chunks"] = len(fds)
        ev["imported"].wait(120)
        out["free_mapped_GB"] = round(_settle(torch, dev), 2)
        ev["importer_released"].wait(120)
        out["free_importer_released_GB"] = round(_settle(torch, dev), 2)
        del arena, vm
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        out["free_both_released_GB"] = round(_settle(torch, dev), 2)
        out["vmm_live"] = list(H.vmm_live())
        ev["exporter_released"].set()
        ev["importer_exited"].wait(120)
        time.sleep(1.0)
        out["free_importer_exited_GB"] = round(_settle(torch, dev), 2)
        out["base_GB"] = round(base, 2)
        out["arena_GB"] = round(n / 1e9, 2)
        out["leak_both_released_GB"] = round(base - out["free_both_released_GB"], 2)
        out["leak_after_importer_exit_GB"] = round(base - out["free_importer_exited_GB"], 2)
        q.put(out)
    else:
        ev["listening"].wait(120)
        with socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET) as c:
            c.connect(name)
            fds = []
            while True:
                _, got, _, _ = socket.recv_fds(c, 1, 200)
                fds += got
                if len(got) < 200:
                    break
            m = H.vmm_import(fds, 512 << 20, 0)
            for fd in fds:
                os.close(fd)
            c.sendall(b"k")
        t = from_dlpack(m.dlpack(n))
        ok = int(t[:16].cpu()[0]) == 7 and int(t[n - 16:].cpu()[0]) == 7
        ev["imported"].set()
        time.sleep(1.0)
        del t, m
        gc.collect()
        torch.cuda.synchronize()
        ev["importer_released"].set()
        ev["exporter_released"].wait(120)
        q.put({"importer_read_ok": ok, "importer_vmm_live": list(H.vmm_live())})
        ev["importer_exited"].set()  # (set just before the process ends; rank 0 waits 1 s more)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ev = {k: ctx.Event() for k in ("listening", "imported", "importer_released", "exporter_released", "importer_exited")}
    port = os.getpid()
    ps = [ctx.Process(target=worker, args=(r, port, a.gb, q, ev)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=400) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    rec = {}
    for r in res:
        rec.update(r)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
