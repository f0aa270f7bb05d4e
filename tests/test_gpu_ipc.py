"""The `ipc` / `xgmi` exchanges on a real GPU: two ranks map each other's HBM arena (HIP IPC over
dmabuf) and pull their peer's regions with DMA copies (`ipc`) or the K8 gather kernel (`xgmi`).  Both ranks share the box's one GPU (gloo carries
the control messages; RCCL refuses two ranks on one device), which exercises the handle exchange,
the per-round readiness (GPU-side ready counters, or the host barrier with ZEST_IPC_SIGNALS=0) and the
copy streams; xGMI bandwidth is measured by bench.py on the 8-GPU node."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rank(rank, port, q, mode, alloc="vmm", signals="1"):
    import faulthandler
    import sys

    import torch.distributed as dist
    faulthandler.dump_traceback_later(150, exit=True, file=sys.stderr)  # a stack instead of a silent hang
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZEST_IPC_SIGNALS=signals)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from zest_amd import ops
        from zest_amd.engine import DevicePuller
        from zest_amd.synthetic import SyntheticWorld
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        w = SyntheticWorld("llama-tiny", seed=11, mode="random", max_xorb_bytes=1 << 20)
        arena = ops.vmm_empty(w.arena_bytes, dev) if alloc == "vmm" else ops.padded_empty(w.arena_bytes, dev)
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
        q.put((rank, ok, bool(same), p.n_rounds, p.bytes_received, p.xchg.signaled))
        dist.barrier()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, False, repr(e), 0, 0, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,alloc,signals", [("ipc", "vmm", "1"), ("xgmi", "vmm", "1"), ("xgmi", "torch", "1"),
                                                ("ipc", "vmm", "0"), ("xgmi", "vmm", "0")])
def test_ipc_exchange_two_ranks_one_gpu(mode, alloc, signals):
    """vmm: the arena is a HIP VMM mapping shared through dmabuf fds (what bench.py uses); torch: a
    caching-allocator tensor shared with hipIpcGetMemHandle (small arenas only, see engine.py).
    signals=1: the exchanges wait on the GPU for the owners' shared ready counters; 0: host event
    synchronize + host barrier per round."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + 50 * (mode == "xgmi") + 100 * (alloc == "torch") + 150 * (signals == "0") + os.getpid() % 50
    procs = [ctx.Process(target=_rank, args=(r, port, q, mode, alloc, signals)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, ok, equal, rounds, recv, signaled in res:
        assert ok is True and equal is True, res
        assert rounds > 1 and recv > 0
        assert signaled is (signals == "1"), res


def _signals_child(path, q):
    """One process, two mappings of one shared page: a stream gated by hipStreamWaitValue32 runs
    only once the counter reaches the value (not before, not at a smaller value), and set_after
    stores a counter stream-ordered behind earlier work."""
    import faulthandler
    import sys
    import time
    faulthandler.dump_traceback_later(60, exit=True, file=sys.stderr)
    try:
        from zest_amd import ops
        H = ops.hip()
        torch.cuda.set_device(0)
        if not H.can_stream_wait_value(0):
            q.put("unsupported")
            return
        a = H.signals_open(path, 2, True, 0)
        b = H.signals_open(path, 2, False, 0)
        os.unlink(path)
        x = torch.zeros(4, device="cuda:0")
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            a.wait_on(1, 5, st.cuda_stream)
            x.fill_(7)
            ev = torch.cuda.Event()
            ev.record(st)
        time.sleep(0.2)
        early = ev.query()
        b.store(1, 4)
        time.sleep(0.2)
        below = ev.query()
        b.store(1, 5)
        t0 = time.time()
        while not ev.query() and time.time() - t0 < 10:
            time.sleep(0.005)
        released = ev.query()
        ok_x = released and float(x[0].item()) == 7.0
        other = torch.cuda.Stream()
        y = torch.randn(2048, 2048, device="cuda:0")
        with torch.cuda.stream(other):
            for _ in range(20):
                y = y @ y.T / 2048.0
            a.set_after(0, 1, other.cuda_stream)
        with torch.cuda.stream(st):
            a.wait_on(0, 1, st.cuda_stream)
            ev2 = torch.cuda.Event()
            ev2.record(st)
        t0 = time.time()
        while not ev2.query() and time.time() - t0 < 10:
            time.sleep(0.005)
        q.put((early, below, released, ok_x, ev2.query(), b.value(0), b.value(1)))
    except Exception as e:  # noqa: BLE001
        q.put(repr(e))


def test_peer_signals_gate_streams():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = f"/dev/shm/zest-sig-test-{os.getpid()}"
    p = ctx.Process(target=_signals_child, args=(path, q))
    p.start()
    try:
        got = q.get(timeout=120)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
        if os.path.exists(path):
            os.unlink(path)
    if got == "unsupported":
        pytest.skip("hipStreamWaitValue32 unsupported on this device")
    assert got == (False, False, True, True, True, 1, 5), got


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


def _big_rank(rank, port, q, gib):
    import faulthandler
    import sys

    import torch.distributed as dist
    faulthandler.dump_traceback_later(150, exit=True, file=sys.stderr)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from zest_amd import ops
        from zest_amd.engine import map_peer_arenas
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        n = int(gib * (1 << 30))
        arena = ops.vmm_empty(n, dev)
        arena.fill_(rank + 1)  # written by a kernel before the export (that made IPC imports hang)
        arena[n - 1] = 100 + rank
        torch.cuda.synchronize()
        m = map_peer_arenas(arena, rank, 2, deadline_s=60)
        peer = m.peers[1 - rank] if m is not None else None
        got = None
        if peer is not None:
            got = (peer.numel(), int(peer[0].item()), int(peer[n // 2].item()), int(peer[n - 1].item()))
        q.put((rank, got))
        dist.barrier()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_vmm_maps_a_large_written_arena():
    """A 6 GiB kernel-written arena per rank, mapped by the sibling rank through the VMM path
    (hipIpcOpenMemHandle of a >= 2 GiB allocation hung on this box)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29950 + os.getpid() % 40
    gib = 6
    procs = [ctx.Process(target=_big_rank, args=(r, port, q, gib)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    n = gib << 30
    assert res == [(0, (n, 2, 2, 101)), (1, (n, 1, 1, 100))], res
