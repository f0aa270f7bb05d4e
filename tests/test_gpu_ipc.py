"""The `ipc` / `xgmi` exchanges on a real GPU: two ranks map each other's HBM arena (HIP IPC over
dmabuf) and pull their peer's regions with DMA copies (`ipc`) or the K8 gather kernel (`xgmi`).  Both ranks share the box's one GPU (gloo carries
the control messages; RCCL refuses two ranks on one device), which exercises the handle exchange,
the per-round host barrier and the copy streams; xGMI bandwidth is measured by bench.py on the
8-GPU node."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rank(rank, port, q, mode):
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
        p.exchange = mode
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


@pytest.mark.parametrize("mode", ["ipc", "xgmi"])
def test_ipc_exchange_two_ranks_one_gpu(mode):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + 50 * (mode == "xgmi") + os.getpid() % 50
    procs = [ctx.Process(target=_rank, args=(r, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, ok, equal, rounds, recv in res:
        assert ok is True and equal is True, res
        assert rounds > 1 and recv > 0


def test_peer_gather_kernel_segments():
    """K8 on local buffers: several segments of odd sizes and offsets (head / vector body / tail
    paths), one launch, byte-exact against torch copies; untouched bytes stay untouched."""
    from zest_amd import ops
    H = ops.hip()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(5)
    src = torch.randint(0, 256, (3 << 20,), dtype=torch.uint8, generator=g).to(dev)
    dst = torch.zeros_like(src)
    segs = [(0, 1), (5, 17), (33, 4096 + 7), (100003, 1 << 20), (2 << 20, (1 << 20) - 13), (3000, 0)]
    H.peer_gather([src.data_ptr() + o for o, _ in segs], [dst.data_ptr() + o for o, _ in segs],
                  [n for _, n in segs], torch.cuda.current_stream().cuda_stream)
    want = torch.zeros_like(src)
    for o, n in segs:
        want[o:o + n] = src[o:o + n]
    torch.cuda.synchronize()
    assert torch.equal(dst, want)
    with pytest.raises(ValueError):
        H.peer_gather([src.data_ptr() + 1], [dst.data_ptr()], [10], 0)
