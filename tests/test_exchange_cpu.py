"""zest_amd.parallel.exchange.RoundExchange on gloo CPU groups: every strategy replicates uneven
per-rank regions (empty ones included) into every rank's arena, on the whole job and on a subgroup
(peers addressed by their global ranks), the all-gather buffers grow when a later round needs a
bigger slab, and autotune's pick is cached per process."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from e2e_util import free_port


def _fill(arena, regions, rank, seed):
    lo, hi = regions[rank]
    if hi > lo:
        g = torch.Generator().manual_seed(seed * 1000 + rank)
        arena[lo:hi] = torch.randint(0, 256, (hi - lo,), dtype=torch.uint8, generator=g)


def _want(n, regions, seed):
    out = torch.zeros(n, dtype=torch.uint8)
    for r in range(len(regions)):
        _fill(out, regions, r, seed)
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from zest_amd.parallel import exchange as X
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1 << 16
        rounds = [[(0, 5000), (5000, 5001), (7000, 9000)],     # uneven
                  [(10000, 10000), (20000, 30000), (30000, 30100)],  # rank 0 sends nothing
                  [(40000, 65536), (0, 0), (100, 200)]]          # a bigger slab later (allgather growth)
        res = {}
        for mode in ("p2p", "bcast", "allgather"):
            arena = torch.zeros(n, dtype=torch.uint8)
            xc = X.RoundExchange(arena, rank, world, None, mode, gather_capacity=2000)
            for k, regs in enumerate(rounds):
                _fill(arena, regs, rank, k)
                for w in xc.exchange(regs):
                    w.wait()
            want = torch.zeros(n, dtype=torch.uint8)
            for k, regs in enumerate(rounds):
                want_k = _want(n, regs, k)
                for lo, hi in regs:
                    want[lo:hi] = want_k[lo:hi]
            res[mode] = bool(torch.equal(arena, want))
        # a subgroup of global ranks 1 and 2: peers are addressed by global rank
        sub = dist.new_group(ranks=[1, 2])
        if rank in (1, 2):
            me = dist.get_rank(sub)
            arena = torch.zeros(4096, dtype=torch.uint8)
            regs = [(0, 1000), (1000, 3000)]
            xc = X.RoundExchange(arena, me, 2, sub, "p2p")
            _fill(arena, regs, me, 7)
            for w in xc.exchange(regs):
                w.wait()
            res["subgroup_p2p"] = bool(torch.equal(arena[:3000], _want(4096, regs, 7)[:3000]))
        # autotune: every rank picks the same mode, cached for the next pull of that shape
        arena = torch.zeros(n, dtype=torch.uint8)
        xc = X.RoundExchange(arena, rank, world, None, "p2p")
        t = xc.autotune(rounds[:2], modes=("p2p", "bcast", "allgather"))
        res["tuned"] = (xc.mode, sorted(t), X.tuned_mode(world, "gloo", False))
        # GPU-side readiness needs peer-mapped arenas: on a CPU group it stays off, the exchange
        # keeps its host path, and a seq handed to exchange() is ignored
        res["signals"] = (xc.enable_signals(), xc.signaled)
        xc.order_after(None)  # no exchange streams: a no-op
        arena = torch.zeros(n, dtype=torch.uint8)
        xc = X.RoundExchange(arena, rank, world, None, "bcast")
        _fill(arena, rounds[0], rank, 0)
        for w in xc.exchange(rounds[0], seq=5):
            w.wait()
        res["seq_ignored"] = bool(torch.equal(arena[:9000], _want(n, rounds[0], 0)[:9000]))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_round_exchange_modes_subgroup_and_autotune():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(3):
        assert res[r]["p2p"] and res[r]["bcast"] and res[r]["allgather"], res[r]
    assert res[1]["subgroup_p2p"] and res[2]["subgroup_p2p"]
    picks = {res[r]["tuned"][0] for r in range(3)}
    assert len(picks) == 1
    for r in range(3):
        mode, timed, cached = res[r]["tuned"]
        assert timed == ["allgather", "bcast", "p2p"] and cached == mode
    for r in range(3):
        assert res[r]["signals"] == (False, False), res[r]
        assert res[r]["seq_ignored"], res[r]
