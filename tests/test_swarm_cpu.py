"""Multi-process intra-node swarm on CPU (gloo): every rank ends with the full, verified model.

This is the CPU rehearsal of the RCCL path (bench.py / zest_amd.engine): same planner, same
per-round peer-to-peer exchange (batch_isend_irecv), same chunk-hash all-reduce + Merkle check.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world_size, port, model, result_q, seeders=None, exchange="p2p"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from zest_amd.engine import DevicePuller
        from zest_amd.synthetic import SyntheticWorld
        w = SyntheticWorld(model, seed=3, mode="random", max_xorb_bytes=256 << 10)
        contents = w.build_on_host()
        arena = torch.zeros(w.arena_bytes + 4096, dtype=torch.uint8)[: w.arena_bytes]
        p = DevicePuller(w, arena, rank, world_size, round_bytes=512 << 10, seeders=seeders)
        p.build_origin_host(contents)
        if exchange == "auto":
            p.autotune_exchange()
        else:
            p.exchange = exchange
        for _ in range(2):
            arena.zero_()
            p.step()
            p.check()
        ok = all(arena[f.arena_off:f.arena_off + f.size].numpy().tobytes() == contents[f.path] for f in w.xet_files)
        result_q.put((rank, ok, p.bytes_received, p.bytes_ingested, w.model_bytes, p.exchange))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size", [2, 3])
def test_cpu_swarm_full_replication(world_size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world_size * 7 + os.getpid() % 100
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, "llama-tiny", q)) for r in range(world_size)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, *_ in res)
    total_in = sum(r[3] for r in res)
    model = res[0][4]
    # every rank ingests ~1/N from the origin and receives the rest from peers
    assert total_in < model * 1.01 + 8 * 4096
    for _, _, recv, ing, m, _x in res:
        assert recv > 0 and recv < m


def test_cpu_seeder_leecher():
    """BASELINE config 2 shape: 1 seeder ingests everything from the origin, the leechers receive
    the whole model from it (P2P ratio 100 % for them)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 100
    procs = [ctx.Process(target=_worker, args=(r, 3, port, "llama-tiny", q, 1)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, *_ in res)
    model = res[0][4]
    assert res[0][2] == 0 and res[0][3] > 0            # seeder: everything from the origin
    for _, _, recv, ing, m, _x in res[1:]:
        assert ing == 0 and recv == m                   # leechers: everything from the seeder


@pytest.mark.parametrize("exchange", ["bcast", "allgather", "auto"])
def test_cpu_swarm_exchange_modes(exchange):
    """The alternative replication strategies (coalesced broadcasts, equal-slab all-gather +
    unpack) and the setup-time autotuner give the same fully verified replica on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + 11 * ["bcast", "allgather", "auto"].index(exchange) + os.getpid() % 100
    procs = [ctx.Process(target=_worker, args=(r, 3, port, "llama-tiny", q, None, exchange)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, *_ in res)
    chosen = {r[5] for r in res}
    assert len(chosen) == 1, chosen  # all ranks agree
    if exchange != "auto":
        assert chosen == {exchange}


def _corrupt_worker(rank, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from zest_amd import ops
        from zest_amd.engine import DevicePuller
        from zest_amd.synthetic import SyntheticWorld

        class Flaky(DevicePuller):
            """Flips one received byte on rank 0 before it is hashed (a bad link / faulty peer)."""

            def _hash_received(self, k, works):
                for w in works:
                    w.wait()
                if self.rank == 0 and k == 0 and self.recv_runs[0]:
                    c0, _ = self.recv_runs[0][0]
                    self.arena[int(self.world.chunk_off[c0]) + 7] ^= 1
                return super()._hash_received(k, [])

        w = SyntheticWorld("llama-tiny", seed=3, mode="random", max_xorb_bytes=256 << 10)
        contents = w.build_on_host()
        arena = torch.zeros(w.arena_bytes + 4096, dtype=torch.uint8)[: w.arena_bytes]
        p = Flaky(w, arena, rank, 2, round_bytes=512 << 10)
        p.build_origin_host(contents)
        p.step()
        try:
            p.check()
            result_q.put((rank, "passed"))
        except ops.IngestError as e:
            result_q.put((rank, f"detected {e.code}"))
    finally:
        dist.destroy_process_group()


def test_cpu_swarm_detects_corrupt_transfer():
    """Every rank hashes what it received itself: one flipped byte on rank 0 fails the Merkle check,
    and the error word is all-reduced so both ranks stop."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29760 + os.getpid() % 100
    procs = [ctx.Process(target=_corrupt_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1].split()[0] for r in res] == ["detected", "detected"], res


def test_cpu_swarm_eight_ranks_autotuned():
    """The round-end scaling bench's shape (8 ranks, one per GPU, exchange autotuned) rehearsed on
    gloo: every rank verifies the full model, all agree on the exchange mode, ingest totals 1x."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + os.getpid() % 100
    procs = [ctx.Process(target=_worker, args=(r, 8, port, "llama-tiny", q, None, "auto")) for r in range(8)]
    for p in procs:
        p.start()
    res = [q.get(timeout=400) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, *_ in res)
    assert len({r[5] for r in res}) == 1
    model = res[0][4]
    assert sum(r[3] for r in res) < model * 1.01 + 8 * 4096


def test_round_plan_taper_covers_every_term_once():
    """Tapered rounds (small head and tail rounds, full rounds <= round_bytes) partition each rank's
    terms in order, identically shaped on every rank."""
    from types import SimpleNamespace

    from zest_amd.engine import plan_rank_terms, round_weights, split_rounds

    # the planners read only the terms' byte sizes: 3000 terms of 8-128 KiB
    T = np.zeros(3000, dtype=[("ulen", np.int64)])
    T["ulen"] = np.random.default_rng(5).integers(8 << 10, 128 << 10, len(T))
    w = SimpleNamespace(terms=T)
    for n_ranks in (1, 3):
        shares = plan_rank_terms(w, n_ranks)
        biggest = max(int(T["ulen"][a:b].sum()) for a, b in shares)
        rb = biggest // 12
        weights = round_weights(biggest, rb)
        assert weights[:2] == [0.25, 0.5] and weights[-3:] == [0.5, 0.25, 0.125]
        assert sum(weights) * rb >= biggest
        for a, b in shares:
            rounds = split_rounds(w, a, b, weights)
            assert len(rounds) == len(weights)
            assert rounds[0][0] == a and rounds[-1][1] == b
            assert all(r0[1] == r1[0] for r0, r1 in zip(rounds, rounds[1:]))
            sizes = [int(T["ulen"][x:y].sum()) for x, y in rounds]
            full = sum(sizes[2:-3]) / max(1, len(sizes) - 5)
            assert sizes[0] < full and sizes[-1] < full
    assert round_weights(3 << 20, 1 << 20) == [1.0] * 3          # short plans are not tapered
    assert round_weights(40 << 20, 1 << 20, taper=False) == [1.0] * 40


def test_arena_in_use_counts_views():
    """swarm_pull's automatic arena reuse only takes a kept arena when no tensor of the earlier pull
    still views it (storage reference count beyond the cached tensor)."""
    import torch

    from zest_amd.parallel.swarm_pull import _arena_in_use, _storage_refs
    base = torch.empty(1 << 16, dtype=torch.uint8)
    full = base[: 1 << 15]
    del base
    entry = (full, None, _storage_refs(full))  # as swarm_pull keeps it
    assert not _arena_in_use(entry)
    views = {"a": full[:100].view(torch.int32), "b": full[4096:8192]}
    assert _arena_in_use(entry)
    del views
    assert not _arena_in_use(entry)


def test_staging_slot_bytes_by_world():
    """Round-synchronous device swarm pulls: N = 1 keeps its staging slots, every N > 1 takes a
    quarter round (round 5's per-world exception for 4 and 8 ranks answered a stall that was the
    hash-table race, docs/ARCHITECTURE.md 16.2), never below 64 MiB and never above the configured
    size."""
    from zest_amd.parallel.swarm_pull import staging_slot_bytes
    gib, mib = 1 << 30, 1 << 20
    assert staging_slot_bytes(gib, gib, 1) == gib
    assert staging_slot_bytes(gib, gib, 2) == 256 * mib
    assert staging_slot_bytes(gib, gib, 4) == 256 * mib
    assert staging_slot_bytes(gib, gib, 8) == 256 * mib
    assert staging_slot_bytes(gib, 128 * mib, 2) == 64 * mib
    assert staging_slot_bytes(128 * mib, 4 * gib, 8) == 128 * mib


def test_agree_thread_finishes_in_order_and_hands_errors_back():
    """_AgreeThread (the streamed pull's agreements): rounds are finished in submission order on the
    thread; the first error stops the processing, later rounds are skipped, and raise_error()
    re-raises it on the pulling thread; close(abandon=True) skips rounds not started."""
    from zest_amd.parallel.swarm_pull import _AgreeThread

    class Sw:
        cuda = False
        device = torch.device("cpu")

        def __init__(self, fail_at=None):
            self.done, self.fail_at = [], fail_at

        def _finish_agree(self, ag):
            if ag == self.fail_at:
                raise RuntimeError(f"round {ag} failed")
            self.done.append(ag)

    sw = Sw()
    t = _AgreeThread(sw)
    for k in range(20):
        t.put(k)
    t.close()
    t.raise_error()
    assert sw.done == list(range(20))

    sw = Sw(fail_at=5)
    t = _AgreeThread(sw)
    for k in range(10):
        t.put(k)
    t.close()
    assert sw.done == [0, 1, 2, 3, 4]
    with pytest.raises(RuntimeError, match="round 5 failed"):
        t.raise_error()

    import threading
    gate = threading.Event()

    class Slow(Sw):
        def _finish_agree(self, ag):
            gate.wait(5)
            super()._finish_agree(ag)

    sw = Slow()
    t = _AgreeThread(sw)
    for k in range(5):
        t.put(k)
    t.abandon = True  # (what close(abandon=True) sets before it joins)
    gate.set()
    t.close(abandon=True)
    assert len(sw.done) <= 1  # the round in progress may finish; the queued ones are skipped
