"""The fd exchange behind the VMM peer mapping (zest_amd.parallel.exchange._import_vmm_peers), on CPU: 3 gloo ranks,
each "arena" exported as memfds whose bytes name the owner and the chunk; every rank must import
every peer's chunks, in order, through the abstract-socket + SCM_RIGHTS protocol.  The HIP side
(hipMemImportFromShareableHandle + mapping) runs in tests/test_gpu_ipc.py."""
import os

import torch


class _FakeMapping:
    def __init__(self, rank=None, n_chunks=0, chunk=4096, content=None):
        self.rank, self.n_chunks, self.chunk, self.content = rank, n_chunks, chunk, content or []

    def export_fds(self):
        fds = []
        for k in range(self.n_chunks):
            fd = os.memfd_create(f"chunk{k}")
            os.write(fd, f"{self.rank}:{k}".encode())
            fds.append(fd)
        return fds

    def dlpack(self, nbytes):
        return torch.zeros(nbytes, dtype=torch.uint8).__dlpack__()


class _FakeHip:
    def vmm_import(self, fds, chunk, device):
        return _FakeMapping(content=[os.pread(fd, 32, 0).decode() for fd in fds], chunk=chunk)


class _Dev:
    index = 0


class _Arena:
    device = _Dev()


class _SlowHip(_FakeHip):
    """Rank 0's imports stall past the whole mapping budget."""

    def vmm_import(self, fds, chunk, device):
        import time
        time.sleep(4.0)
        return super().vmm_import(fds, chunk, device)


def _rank(rank, world, port, q, budget=30.0, slow_rank=None):
    import torch.distributed as dist

    from zest_amd import ops
    from zest_amd.parallel import exchange as engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops.hip = (lambda: _SlowHip()) if rank == slow_rank else (lambda: _FakeHip())
        engine._vmm_mark = lambda *a: None  # the pad sentinel read-back needs a GPU (test_gpu_ipc.py)
        engine._vmm_check = lambda *a: True
        n_chunks = 3 + rank  # ranks own different chunk counts
        vm = _FakeMapping(rank, n_chunks)
        mine = ("vmm", f"tok{port}" if rank == 0 else "ignored", 4096, n_chunks, 100 + rank)
        objs = [None] * world
        dist.all_gather_object(objs, mine)
        hg = dist.new_group(backend="gloo")
        peers = [None] * world
        import time
        t0 = time.monotonic()
        ok = engine._import_vmm_peers(_Arena(), vm, objs, rank, world, hg, peers, budget)
        got = {p: (t.numel(), t._zest_vmm.content) for p, t in enumerate(peers) if t is not None}
        q.put((rank, ok, got, time.monotonic() - t0))
    except Exception as e:  # noqa: BLE001
        q.put((rank, False, repr(e), 0.0))
    finally:
        dist.destroy_process_group()


def test_vmm_fd_exchange_three_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 3, 29900 + os.getpid() % 80
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    for rank, ok, got, _ in res:
        assert ok is True, (rank, got)
        assert sorted(got) == [p for p in range(world) if p != rank]
        for p, (numel, content) in got.items():
            assert numel == 100 + p
            assert content == [f"{p}:{k}" for k in range(3 + p)]


def test_vmm_mapping_budget_covers_all_turns():
    """The deadline bounds the mapping as a whole: rank 0's import turn stalls past the 2 s budget,
    so ranks 1 and 2 skip theirs; every rank reports failure (the caller falls back to RCCL) well
    before per-turn deadlines would have added up, and no serving thread keeps a rank waiting."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 3, 29980 + os.getpid() % 15
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, 2.0, 0)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    for rank, ok, got, dt in res:
        assert ok is False, (rank, got)
        assert dt < 15.0, (rank, dt)
