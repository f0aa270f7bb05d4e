"""The `ipc` exchange on a real GPU: two ranks map each other's HBM arena (HIP IPC over dmabuf)
and pull their peer's regions with DMA copies.  Both ranks share the box's one GPU (gloo carries
the control messages; RCCL refuses two ranks on one device), which exercises the handle exchange,
the per-round host barrier and the copy streams; xGMI bandwidth is measured by bench.py on the
8-GPU node."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rank(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from zest_amd import ops
        from zest_amd.engine import DevicePuller
        from zest_amd.synthetic import SyntheticWorld
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        w = SyntheticWorld("llama-tiny", seed=11, mode="random", max_xorb_bytes=1 << 20)
        arena = ops.padded_empty(w.arena_bytes, dev)
        w.generate_on_device(arena)
        w.build_on_device(arena)
        want = arena.clone()
        p = DevicePuller(w, arena, rank, 2, round_bytes=1 << 20)
        p.build_origin()
        ok = p.enable_ipc()
        p.exchange = "ipc"
        for _ in range(2):
            arena.fill_(0xA5)
            p.err.zero_()
            p.step()
            torch.cuda.synchronize()
            p.check()
        same = all(torch.equal(arena[f.arena_off:f.arena_off + f.size], want[f.arena_off:f.arena_off + f.size])
                   for f in w.xet_files)  # the alignment gaps between files are not part of any term
        q.put((rank, ok, bool(same), p.n_rounds, p.bytes_received))
        dist.barrier()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, False, repr(e), 0, 0))
    finally:
        dist.destroy_process_group()


def test_ipc_exchange_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + os.getpid() % 100
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, ok, equal, rounds, recv in res:
        assert ok is True and equal is True, res
        assert rounds > 1 and recv > 0
