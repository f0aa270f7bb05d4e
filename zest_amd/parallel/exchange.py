"""Intra-node piece exchange: replicate each rank's freshly ingested arena region to
every other GPU of the node, the GPUs acting as BitTorrent peers for each other.

One `RoundExchange` per arena.  Every round, each rank owns one contiguous region [lo, hi) of the
arena (its share of the round's terms, already decoded and hashed in place); `exchange(regions)`
makes every rank's region appear at the same offsets of every peer's arena.  Strategies:

* ``p2p``       batch_isend_irecv: each owner sends its region to every peer (N-1 pairs).
* ``bcast``     uneven all_gather straight into the arena views (RCCL: one coalesced group of N
                broadcasts, zero copy).
* ``allgather`` equal-size slabs through all_gather_into_tensor into a double-buffered gather buffer,
                then a D2D unpack on a side stream (RCCL's ring allgather).
* ``ipc``       no collective: every rank maps its peers' arenas (HIP VMM dmabuf fds, `map_peer_arenas`)
                and pulls their regions with DMA copies, one stream per peer group, so the copies of
                all 7 peers run over their own xGMI links at once.
* ``xgmi``      same mapping, one K8 kernel (csrc/gpu/xgmi.hip) reads every peer's region with 16-byte
                loads from all CUs: every link is read concurrently from a single launch.

Which is fastest depends on RCCL's channel/link mapping over the xGMI mesh, so `autotune` times them
on the machine (setup, untimed) and keeps the fastest; the choice is cached per process
(`tuned_mode`) so later pulls of the same shape skip the sweep.  Used by the bench engine
(zest_amd.engine.DevicePuller) and by the public multi-GPU pull (zest_amd.parallel.swarm_pull).

Fault injection (tests): ZEST_VMM_FAULT=import makes every peer import raise,
=sentinel makes the mapping's read-back check fail (both: the mapping is refused and the caller
falls back to an RCCL exchange), =gather corrupts the first bytes of every region a peer-mapped
exchange receives (the receiver's hash check catches it and the caller drops to ``p2p``).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import torch

from .. import ops

EXCHANGE_MODES = ("p2p", "bcast", "allgather", "ipc", "xgmi")
PEER_MAPPED_MODES = ("ipc", "xgmi")  # need enable_ipc()


def vmm_fault() -> str:
    return os.environ.get("ZEST_VMM_FAULT", "")


class StreamJoin:
    """Work-like handle: wait() orders the current stream after everything queued on `stream`."""

    def __init__(self, stream):
        self.event = torch.cuda.Event()
        self.event.record(stream)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)


# Streams created once per process and role.  torch hands out streams from a round-robin pool and
# HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4 here); a second DevicePuller in
# the same process drew other pool streams, its two compute lanes shared a queue, and its pull ran
# at 52.9 instead of 56.9 GB/s (profiles/bench70b_modes_r3.md).  Reusing the first puller's streams
# keeps the lane/copy layout that was measured.
_STREAMS: dict = {}


def role_stream(device: torch.device, role: str, priority: int = 0):
    key = (device.index, role)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(device, priority=priority)
    return _STREAMS[key]


# ----------------------------------------------------------------------------------------------
# Peer arena mapping (HIP VMM dmabuf fds, or HIP IPC handles for small torch allocations)
# ----------------------------------------------------------------------------------------------
@dataclass
class PeerArenas:
    """Every peer's arena mapped into this process (``peers[rank]`` is None), plus the gloo group the
    ``ipc`` exchange's host barriers use.  ``signals`` / ``sig_sent``: the ready-counter page shared
    over these ranks (RoundExchange.enable_signals) and this rank's last counter value, kept with the
    mapping so later exchanges over it (the next pull reusing the arena) reuse the page."""
    arena: "torch.Tensor"
    peers: list
    host_group: object
    signals: object = None
    sig_sent: int = 0


def map_peer_arenas(arena, rank: int, n_ranks: int, group=None, deadline_s: float | None = None):
    """Collective: share this rank's arena with every peer and map every peer's.  Returns a
    :class:`PeerArenas`, or None unless every rank mapped every peer (MIN-reduced).

    Arenas from :func:`ops.vmm_empty` go through the HIP VMM path: each rank serves its chunks'
    dmabuf fds on an abstract Unix socket, and the peers import and map them contiguously
    (:func:`_import_vmm_peers`).  Other arenas use HIP IPC handles (``reduce_tensor``), imported one
    rank at a time; on the MI355X box hipIpcOpenMemHandle of a >= 2 GiB allocation hung (64-512 MiB
    imports took < 2 ms, profiles/ipc_import_sizes_r3.txt), so that path is for small arenas.
    ``deadline_s`` (default ``ZEST_IPC_DEADLINE`` = 60 s) bounds the imports: a rank whose imports do
    not return in time reports failure, and the caller falls back to an RCCL exchange.  On the VMM
    path the deadline covers all the ranks' import turns together."""
    import threading
    import uuid

    import torch.distributed as dist
    from torch.multiprocessing.reductions import reduce_tensor
    if arena.device.type != "cuda" or n_ranks == 1:
        return None
    if deadline_s is None:
        deadline_s = float(os.environ.get("ZEST_IPC_DEADLINE", "60"))
    vm = ops.vmm_mapping(arena)
    if vm is not None:
        mine = ("vmm", uuid.uuid4().hex, vm.chunk, vm.n_chunks, arena.numel())
    else:
        try:
            mine = ("ipc", reduce_tensor(arena))
        except Exception:
            mine = None
    objs = [None] * n_ranks
    dist.all_gather_object(objs, mine, group=group)
    # host-only barrier (gloo): does not wait on this rank's GPU streams like an RCCL barrier
    host_group = dist.new_group(backend="gloo") if group is None else \
        dist.new_group(ranks=dist.get_process_group_ranks(group), backend="gloo", use_local_synchronization=True)
    peers = [None] * n_ranks
    ok = 1
    if all(o is not None and o[0] == "vmm" for o in objs):
        ok = int(_import_vmm_peers(arena, vm, objs, rank, n_ranks, host_group, peers, deadline_s))
    elif all(o is not None and o[0] == "ipc" for o in objs):
        # One rank imports at a time: two processes opening each other's large dmabuf handles at
        # the same moment deadlocked inside hipIpcOpenMemHandle; an exporter idle in a barrier
        # answers at once.
        for turn in range(n_ranks):
            if turn == rank:
                res: dict = {}

                def imp():
                    try:
                        if vmm_fault() == "import":
                            raise RuntimeError("injected import failure (ZEST_VMM_FAULT=import)")
                        H = ops.hip()
                        for p, o in enumerate(objs):
                            if p != rank:
                                fn, args = o[1]
                                t = fn(*args)
                                if t.device != arena.device and not H.enable_peer_access(t.device.index):
                                    raise RuntimeError(f"no peer access to {t.device}")
                                res[p] = t
                    except Exception as e:  # noqa: BLE001
                        res["error"] = e
                th = threading.Thread(target=imp, daemon=True)
                th.start()
                th.join(deadline_s)
                if th.is_alive() or "error" in res:
                    ok = 0  # a hung import stays parked in its daemon thread; this rank reports failure
                else:
                    for p in range(n_ranks):
                        peers[p] = res.get(p)
            dist.barrier(group=host_group)
    else:
        ok = 0  # some rank could not export (or the ranks disagree on the path)
    flag = torch.tensor([ok], dtype=torch.int32, device=arena.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if not int(flag.item()):
        return None
    return PeerArenas(arena, peers, host_group)


def _vmm_sentinel(token: str, p: int) -> torch.Tensor:
    import hashlib
    return torch.frombuffer(bytearray(hashlib.blake2b(f"{token}:{p}".encode(), digest_size=8).digest()),
                            dtype=torch.uint8)


def _vmm_mark(arena, token: str, rank: int) -> None:
    """8 bytes in the arena's pad (past its logical end, inside the mapping) that every importer
    reads back through its new mapping (:func:`_vmm_check`) before trusting it."""
    st = torch.cuda.current_stream(arena.device)
    mark = _vmm_sentinel(token, rank)
    ops.hip().memcpy_async(arena.data_ptr() + arena.numel(), mark.data_ptr(), 8, st.cuda_stream)
    st.synchronize()


def _vmm_check(t, numel: int, token: str, p: int) -> bool:
    if vmm_fault() == "sentinel":
        return False
    st = torch.cuda.current_stream(t.device)
    got = torch.zeros(8, dtype=torch.uint8)
    ops.hip().memcpy_async(got.data_ptr(), t.data_ptr() + numel, 8, st.cuda_stream)
    st.synchronize()
    return torch.equal(got, _vmm_sentinel(token, p))


_FD_FLOOR = [4096]


def _fresh_fds(fds: list[int]) -> list[int]:
    """Move received fds to numbers this process never used before (F_DUPFD above a rising floor),
    closing the originals: an import must not be told a dmabuf by a recycled fd number
    (ZEST_VMM_FRESH_FDS=1; tools/vmm_leak_probe.py)."""
    import fcntl
    out = []
    for fd in fds:
        try:
            nfd = fcntl.fcntl(fd, fcntl.F_DUPFD_CLOEXEC, _FD_FLOOR[0])
        except OSError:
            out.append(fd)
            continue
        _FD_FLOOR[0] = nfd + 1
        os.close(fd)
        out.append(nfd)
    return out


def _import_vmm_peers(arena, vm, objs, rank, n_ranks, host_group, peers, deadline_s) -> bool:
    """VMM half of :func:`map_peer_arenas`: serve this rank's chunk fds, import every peer's.

    Each rank exports its chunks once (fds) and listens on the abstract Unix socket
    ``zest-vmm-<token>-<rank>`` (token from rank 0, so concurrent jobs on a node do not collide); a
    thread answers every connection with duplicates of those fds (SCM_RIGHTS, <= 200 per message)
    and makes no HIP call.  The ranks then import in turns, one rank at a time, as the IPC path
    does: a process importing while its exporter is itself inside an import is the pattern that
    deadlocked the IPC path, and an idle exporter costs nothing here (16 GiB of chunks mapped in
    22-43 ms, profiles/vmm_ipc_probe_r3.txt)."""
    import socket
    import threading

    import torch.distributed as dist
    from torch.utils.dlpack import from_dlpack

    debug = os.environ.get("ZEST_IPC_DEBUG") == "1"

    def dbg(msg):
        if debug:
            print(f"[vmm rank {rank}] {msg}", flush=True)

    token = objs[0][1]
    try:  # a 141 GB arena is 282 chunk fds, held next to a peer's 282 while they are imported
        import resource
        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        want = 4 * max(o[3] for o in objs) + 256
        if soft != resource.RLIM_INFINITY and soft < want:
            resource.setrlimit(resource.RLIMIT_NOFILE, (want if hard == resource.RLIM_INFINITY else min(want, hard), hard))
    except (ImportError, ValueError, OSError):
        pass
    _vmm_mark(arena, token, rank)
    fds_mine = vm.export_fds()
    dbg(f"exported {len(fds_mine)} chunk fds")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    srv.bind(f"\0zest-vmm-{token}-{rank}")
    srv.listen(n_ranks)
    srv.settimeout(deadline_s * n_ranks)
    served = {"error": None}

    def serve():
        try:
            for _ in range(n_ranks - 1):
                conn, _ = srv.accept()
                with conn:
                    dup = [os.dup(fd) for fd in fds_mine]
                    try:
                        for i in range(0, len(dup), 200):
                            socket.send_fds(conn, [b"z"], dup[i:i + 200])
                        conn.recv(1)  # the importer's ack: it holds its own references now
                    finally:
                        for fd in dup:
                            os.close(fd)
        except Exception as e:  # noqa: BLE001
            served["error"] = e

    res: dict = {}

    def imp():
        try:
            H = ops.hip()
            dev = arena.device.index
            for k in range(1, n_ranks):
                p = (rank + k) % n_ranks
                _, _, chunk, n_chunks, numel = objs[p]
                with socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET) as c:
                    c.settimeout(deadline_s)
                    c.connect(f"\0zest-vmm-{token}-{p}")
                    fds: list[int] = []
                    while len(fds) < n_chunks:
                        _, got, _, _ = socket.recv_fds(c, 1, 200)
                        if not got:
                            raise RuntimeError(f"rank {p} closed the fd stream early")
                        fds += got
                    dbg(f"received {len(fds)} fds from rank {p}; importing")
                    if os.environ.get("ZEST_VMM_FRESH_FDS", "0") == "1":
                        fds = _fresh_fds(fds)
                    try:
                        if vmm_fault() == "import":
                            raise RuntimeError("injected import failure (ZEST_VMM_FAULT=import)")
                        m = H.vmm_import(fds, chunk, dev)
                    finally:
                        for fd in fds:
                            os.close(fd)
                    c.sendall(b"k")
                t = from_dlpack(m.dlpack(numel))
                t._zest_vmm = m
                if not _vmm_check(t, numel, token, p):
                    raise RuntimeError(f"rank {p}'s arena does not read back through the mapping")
                res[p] = t
                dbg(f"mapped rank {p}'s {numel} bytes")
        except Exception as e:  # noqa: BLE001
            res["error"] = e

    st = threading.Thread(target=serve, daemon=True)
    st.start()
    dist.barrier(group=host_group)  # every rank is listening
    # `deadline_s` bounds the whole mapping, not each turn: with 8 ranks and 141 GB arenas a slow
    # import on every turn would otherwise add up past the caller's watchdog (bench.py's "ipc"
    # phase) instead of falling back to RCCL.  A rank whose turn starts after the budget is spent
    # does not import and reports failure; the MIN-reduce in map_peer_arenas then drops the mapping.
    t_end = time.monotonic() + deadline_s
    imported = True
    for turn in range(n_ranks):
        if turn == rank:
            left = t_end - time.monotonic()
            if left <= 0:
                imported = False
                dbg("mapping budget spent before this rank's turn: not importing")
            else:
                it = threading.Thread(target=imp, daemon=True)
                it.start()
                it.join(left)
                imported = not it.is_alive() and "error" not in res
                if "error" in res:
                    dbg(f"import failed: {res['error']}")
        dist.barrier(group=host_group)
    # Every turn is over: a peer that imported has been served and acknowledged, so the serving
    # thread has ended unless some rank skipped its turn; closing the socket ends its accept().
    st.join(1.0)
    complete = not st.is_alive() and served["error"] is None
    srv.close()
    st.join(5.0)
    for fd in fds_mine:
        os.close(fd)
    ok = imported and complete
    if ok:
        for p in range(n_ranks):
            peers[p] = res.get(p)
    return ok


def open_signal_page(group, rank: int, n_slots: int, device):
    """Collective over `group` (gloo): one shared page of `n_slots` 32-bit counters that every rank
    maps and registers with HIP (csrc/bind/hip_signals.cpp), or None on every rank unless every rank
    mapped it and its device can wait on a value (hipStreamWaitValue32)."""
    import uuid

    import torch.distributed as dist
    H = ops.hip()
    dev = device.index or 0

    def agree(v: int) -> int:
        t = torch.tensor([v], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        return int(t.item())
    try:
        ok = int(bool(H.can_stream_wait_value(dev)))
    except Exception:  # noqa: BLE001
        ok = 0
    box = [f"/dev/shm/zest-sig-{uuid.uuid4().hex}" if rank == 0 else None]
    dist.broadcast_object_list(box, src=dist.get_process_group_ranks(group)[0], group=group)
    path = box[0]
    sig = None
    if rank == 0 and ok:
        try:
            sig = H.signals_open(path, n_slots, True, dev)
        except Exception:  # noqa: BLE001
            ok = 0
    ok = agree(ok)  # the page exists (or nobody opens it)
    if ok and rank != 0:
        try:
            sig = H.signals_open(path, n_slots, False, dev)
        except Exception:  # noqa: BLE001
            sig, ok = None, 0
    ok = agree(ok)  # everyone mapped it: the name is no longer needed
    if rank == 0:
        try:
            os.unlink(path)
        except OSError:
            pass
    return sig if ok else None


# ----------------------------------------------------------------------------------------------
# Peer windows: fixed exchange buffers mapped once per process
# ----------------------------------------------------------------------------------------------
@dataclass
class PeerWindows:
    """Every rank's exchange window -- `slots` slots of `slot_bytes` (+ 256 alignment bytes) of HIP
    VMM memory -- mapped into every rank of the group ONCE per process (tools/vmm_oneway_probe.py: the
    HIP runtime keeps a released VMM import alive until the importing process exits, and a re-import
    after a release read the old allocation's bytes, profiles/r6/vmm_release_r6h_r6i/).  The public
    pull's arenas are then ordinary allocations, freed with the caller's tensors, and nothing is
    imported per pull.  ``signals``: 2n counters -- ready[r] (slot r) and read[r] (slot n + r), both
    equal to the window rounds rank r has published / finished reading; ``sent``: this rank's count."""
    window: "torch.Tensor"
    mapped: PeerArenas
    slots: int
    slot_bytes: int
    stride: int
    signals: object = None
    sent: int = 0


_WINDOWS: dict = {}


def window_key(device, group, n_ranks: int) -> tuple:
    import torch.distributed as dist
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(n_ranks))
    return (device.index, ranks)


def peer_windows(device, rank: int, n_ranks: int, group, slot_bytes: int, slots: int):
    """Collective: the group's PeerWindows, created and mapped now -- once per process and group
    (the caller agreed beforehand that some rank lacks usable windows) -- or None when the mapping or
    the counter page cannot be had (the caller then uses an RCCL exchange)."""
    key = window_key(device, group, n_ranks)
    stride = (int(slot_bytes) + 256 + 4095) // 4096 * 4096
    try:
        win = ops.vmm_empty(slots * stride, device)
    except Exception:  # noqa: BLE001
        win = None
    import torch.distributed as dist
    ok = torch.tensor([int(win is not None)], dtype=torch.int64, device=device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if not int(ok.item()):
        return None
    mapped = map_peer_arenas(win, rank, n_ranks, group)
    if mapped is None:
        return None
    sig = open_signal_page(mapped.host_group, rank, 2 * n_ranks, device)
    if sig is None:
        return None
    pw = PeerWindows(win, mapped, int(slots), int(slot_bytes), stride, sig, 0)
    _WINDOWS[key] = pw  # kept for the process: releasing an import would not return its memory
    return pw


# ----------------------------------------------------------------------------------------------
# The exchange
# ----------------------------------------------------------------------------------------------
# Autotuned mode per (world size, backend, arena-mapped) of this process: later pulls skip the sweep.
_TUNED: dict = {}


def tuned_mode(n_ranks: int, backend: str, mapped: bool) -> str | None:
    return _TUNED.get((n_ranks, backend, mapped))


class RoundExchange:
    """Replicates per-round arena regions among the ranks of `group` (see the module docstring)."""

    def __init__(self, arena: torch.Tensor, rank: int, n_ranks: int, group=None, mode: str = "p2p",
                 gather_capacity: int = 0):
        self.arena = arena
        self.device = arena.device
        self.is_cuda = self.device.type == "cuda"
        self.rank, self.n_ranks, self.group = rank, n_ranks, group
        self.mode = mode
        self.times: dict = {}
        self.bytes_moved = 0          # bytes this rank received through exchange() calls
        # host time the peer-mapped modes spend on their ready-event wait and host barrier
        # (the issue path's only host serialization): seconds, and calls
        self.host_wait_s = {"event": 0.0, "barrier": 0.0, "calls": 0}
        self._gather_cap = int(gather_capacity)
        self._gather_bufs = None
        self._gather_n = 0
        self._peer_arenas = None
        self._host_group = None
        self._signals = None          # shared ready counters (enable_signals)
        self._sig_sent = 0            # signal_ready calls so far (= this rank's counter value)
        self._pa = None               # the PeerArenas of enable_ipc
        self._win = None              # PeerWindows of enable_window (peer-mapped modes through windows)

    # -- helpers ------------------------------------------------------------------------------
    def backend(self) -> str:
        import torch.distributed as dist
        return str(dist.get_backend(self.group)).lower()

    def _global_rank(self, r: int) -> int:
        import torch.distributed as dist
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def sync(self):
        if self.is_cuda:
            torch.cuda.synchronize(self.device)

    @property
    def mapped(self) -> bool:
        return self._peer_arenas is not None

    def enable_ipc(self, mapped: "PeerArenas | None" = None) -> bool:
        """Map every peer's arena into this process for the ``ipc`` / ``xgmi`` exchanges.
        ``mapped``: the result of :func:`map_peer_arenas` done earlier (right after the arena was
        allocated); otherwise the mapping is done now.  Collective; True only if every rank mapped
        every peer."""
        if not self.is_cuda or self.n_ranks == 1:
            return False
        if mapped is None:
            mapped = map_peer_arenas(self.arena, self.rank, self.n_ranks, self.group)
        if mapped is None or mapped.arena.data_ptr() != self.arena.data_ptr():
            return False
        self._host_group = mapped.host_group
        self._peer_arenas = mapped.peers
        self._pa = mapped
        self._ipc_streams = [role_stream(self.device, f"ipc{i}") for i in range(min(self.n_ranks - 1, 4))]
        return True

    def enable_window(self, pw: "PeerWindows", resync: int | None = None) -> bool:
        """Peer-mapped exchanges (``ipc`` / ``xgmi``) through the group's PeerWindows instead of
        mapped arenas: per window round the owner copies its region piece into its window slot and
        publishes it (ready counter), the readers copy it out of the owner's window into their own
        arenas and report it read (read counter), which frees the slot for the owner `slots` rounds
        later -- every wait on the GPU.  `resync` (the highest window-round count any rank reached,
        agreed by the caller): every rank's counters continue from there."""
        if not self.is_cuda or self.n_ranks == 1 or pw is None or pw.signals is None:
            return False
        if resync is not None and int(resync) != pw.sent:
            pw.signals.store(self.rank, int(resync))
            pw.signals.store(self.n_ranks + self.rank, int(resync))
            pw.sent = int(resync)
        self._win = pw
        self._host_group = pw.mapped.host_group
        self._peer_arenas = pw.mapped.peers  # (marks the exchange peer-mapped: autotune times ipc / xgmi)
        self._ipc_streams = [role_stream(self.device, f"ipc{i}") for i in range(min(self.n_ranks - 1, 4))]
        self._signal_stream = role_stream(self.device, "signal")
        return True

    def _exchange_window(self, regions, kernel: bool, event=None) -> list:
        pw, H = self._win, ops.hip()
        sig, n, me = pw.signals, self.n_ranks, self.rank
        ss = self._signal_stream
        ss.wait_stream(torch.cuda.current_stream(self.device))
        if event:
            H.stream_wait_event(ss.cuda_stream, int(event))  # the owner's region is written
        size = max((hi - lo for lo, hi in regions), default=0)
        pieces = max(1, -(-size // pw.slot_bytes))

        def piece(r, j):
            lo, hi = regions[r]
            a = lo + j * pw.slot_bytes
            return (a, min(hi, a + pw.slot_bytes)) if a < hi else (0, 0)
        wbase, abase = pw.window.data_ptr(), self.arena.data_ptr()
        streams = self._ipc_streams[:1] if kernel else self._ipc_streams
        fin = streams[0]
        for j in range(pieces):
            k = pw.sent  # window round: the same sequence on every rank
            pw.sent += 1
            slot = k % pw.slots
            if k >= pw.slots:  # every reader finished the slot's previous round
                for r in range(n):
                    if r != me:
                        sig.wait_on(n + r, k - pw.slots + 1, ss.cuda_stream)
            a, b = piece(me, j)
            if b > a:
                H.memcpy_async(wbase + slot * pw.stride + (a & 255), abase + a, b - a, ss.cuda_stream)
            sig.set_after(me, k + 1, ss.cuda_stream)
            segs = []
            for p in range(n):
                pa_, pb = piece(p, j) if p != me else (0, 0)
                if pb > pa_:
                    segs.append((p, self._peer_arenas[p].data_ptr() + slot * pw.stride + (pa_ & 255), abase + pa_,
                                 pb - pa_))
            used = []
            if kernel:
                for p, _, _, _ in segs:
                    sig.wait_on(p, k + 1, fin.cuda_stream)
                for i in range(0, len(segs), 16):
                    part = segs[i:i + 16]
                    H.peer_gather([x[1] for x in part], [x[2] for x in part], [x[3] for x in part], fin.cuda_stream)
            else:
                for i, (p, src, dst, nb) in enumerate(segs):
                    st = streams[i % len(streams)]
                    sig.wait_on(p, k + 1, st.cuda_stream)
                    H.memcpy_async(dst, src, nb, st.cuda_stream)
                    if st is not fin and st not in used:
                        used.append(st)
                for st in used:
                    fin.wait_stream(st)
            if segs:
                self._inject_gather_fault([(sg[0], sg[2] - abase, sg[2] - abase + sg[3]) for sg in segs], fin)
            sig.set_after(n + me, k + 1, fin.cuda_stream)  # this rank has read window round k
        return [StreamJoin(fin)]

    # -- device-side readiness (csrc/bind/hip_signals.cpp) ------------------------------------
    @property
    def signaled(self) -> bool:
        return self._signals is not None

    def enable_signals(self, agreed=None) -> bool:
        """Collective over the mapped ranks: share one page of ready counters (one per rank) so that
        peer-mapped exchanges wait on the GPU (hipStreamWaitValue32 on the owner's counter) instead
        of a host event synchronize + host barrier per round.  Off with ZEST_IPC_SIGNALS=0; False
        (and nothing changes) unless every rank mapped the page and its device can wait on a value."""
        import torch.distributed as dist
        if self._peer_arenas is None or self._host_group is None:
            return False
        if os.environ.get("ZEST_IPC_SIGNALS", "1") == "0":
            return False
        H = ops.hip()
        dev = self.device.index or 0
        g = self._host_group

        def agree(v: int, op=dist.ReduceOp.MIN) -> int:
            t = torch.tensor([v], dtype=torch.int64)
            dist.all_reduce(t, op=op, group=g)
            return int(t.item())

        pa = self._pa
        if agreed is not None and agreed[0] and pa is not None and pa.signals is not None:
            # the caller already agreed (one control all-gather) that every rank keeps this mapping's
            # page, and on the highest counter value any rank reached: no collective here.  Every
            # counter continues from there, so no wait of this pull can be satisfied by an earlier
            # one; no barrier is needed (each rank only raises its own counter, to at most `top`).
            top = int(agreed[1])
            pa.signals.store(self.rank, top)
            pa.sig_sent = top
            self._signals, self._sig_sent = pa.signals, top
            self._signal_stream = role_stream(self.device, "signal")
            return True
        if agree(int(pa is not None and pa.signals is not None)):
            # the mapping's page from an earlier exchange over it (a previous pull): every rank's
            # counter continues from the highest value any rank reached, so a wait of this pull can
            # never be satisfied by an earlier one, whatever the earlier pull left behind
            self.sync()  # no host function of ours may still store an older value
            top = agree(int(pa.sig_sent), dist.ReduceOp.MAX)
            pa.signals.store(self.rank, top)
            pa.sig_sent = top
            dist.barrier(group=g)
            self._signals, self._sig_sent = pa.signals, top
            self._signal_stream = role_stream(self.device, "signal")
            return True
        sig = open_signal_page(g, self.rank, self.n_ranks, self.device)
        if sig is None:
            return False
        self._signals = sig
        self._sig_sent = 0
        if pa is not None:
            pa.signals, pa.sig_sent = sig, 0
        self._signal_stream = role_stream(self.device, "signal")
        return True

    def release_signals(self) -> None:
        """Open every ready counter (0xFFFFFFFF) so that no exchange stream waits any more -- a lost
        rank's counter would never advance -- and stop using the page (the mapping forgets it: its
        sequence is broken).  Copies already queued read whatever the dead owner left; the caller
        re-sends or re-fetches those ranges."""
        if self._win is not None and self._win.signals is not None:
            self._win.signals.release()
            self._win.signals = None  # (the windows stay mapped; the next pull opens a fresh page)
        sig = self._signals
        if sig is None:
            return
        sig.release()
        self._signals = None
        if self._pa is not None and self._pa.signals is sig:
            self._pa.signals = None

    def order_after(self, stream) -> None:
        """With ready counters the exchange streams wait only for the owners' counters, not for this
        rank's host: a caller that writes the receiving regions itself (bench.py's warm-up poisons
        the arena on the main stream before each step) orders the exchange streams after that work
        with this.  (The host-synchronized path got the ordering from its event synchronize.)"""
        for st in getattr(self, "_ipc_streams", ()):
            st.wait_stream(stream)

    def signal_ready(self, stream) -> int:
        """This rank's next region is complete once `stream`'s queued work is: queue the counter
        update behind it (on the signal stream, so `stream` never waits for the host function).
        Returns the sequence number the peers' exchange() must be given for that region.  Every
        rank calls this once per region, in the same order (ranks with empty regions included)."""
        self._sig_sent += 1
        if self._pa is not None:
            self._pa.sig_sent = self._sig_sent
        ss = self._signal_stream
        if stream is not None:
            ss.wait_stream(stream)
        self._signals.set_after(self.rank, self._sig_sent, ss.cuda_stream)
        return self._sig_sent

    def exchange_after(self, regions, event=None, mode: str | None = None) -> list:
        """exchange(regions) once this rank's own region is complete, without a host wait: `event`
        is a raw hipEvent_t recorded after the work writing it (DeviceXetPull.wait_item; None: the
        region is complete on the host, CPU groups, or with the current stream's queued work).
        Peer-mapped modes with ready counters signal after the event and wait for the owners' counters
        on the GPU; without counters the event is host-synchronized and a host barrier follows; the
        RCCL modes issue their collective from a stream ordered after the event.  Every rank calls
        this for every round, in the same order."""
        mode = mode or self.mode
        if not self.is_cuda:
            return self.exchange(regions, mode)
        H = ops.hip()
        cur = torch.cuda.current_stream(self.device)
        if mode in PEER_MAPPED_MODES and self._win is not None:
            regions = [(int(lo), int(hi)) for lo, hi in regions]
            self.bytes_moved += sum(hi - lo for p, (lo, hi) in enumerate(regions) if p != self.rank and hi > lo)
            return self._exchange_window(regions, kernel=(mode == "xgmi"), event=event)
        if mode in PEER_MAPPED_MODES:
            if self._signals is not None:
                ss = self._signal_stream
                ss.wait_stream(cur)
                if event:
                    H.stream_wait_event(ss.cuda_stream, int(event))
                return self.exchange(regions, mode, seq=self.signal_ready(None))
            ready = torch.cuda.Event()
            if event:
                H.stream_wait_event(cur.cuda_stream, int(event))
            ready.record(cur)
            return self.exchange(regions, mode, ready=ready)
        xs = role_stream(self.device, "xissue")
        xs.wait_stream(cur)
        if event:
            H.stream_wait_event(xs.cuda_stream, int(event))
        with torch.cuda.stream(xs):
            return self.exchange(regions, mode)

    # -- one exchange -------------------------------------------------------------------------
    def exchange(self, regions, mode: str | None = None, ready=None, synced: bool = False, seq: int | None = None) -> list:
        """Replicate `regions` ([lo, hi) per rank; empty = that rank sends nothing) to every rank.
        Returns work handles to wait on (stream-ordered on the GPU).

        Peer-mapped modes read the owners' arenas directly, so the owners' regions must be complete:
        with shared ready counters (enable_signals) and `seq` (what every owner's signal_ready
        returned for these regions) the exchange streams wait on the GPU for each owner's counter;
        otherwise `ready` (an event recorded after this rank's region was written) is
        host-synchronized and a host barrier follows; `synced=True` says the caller already
        synchronized every owner (e.g. a control-plane all_gather after blocking fetches) and skips
        both."""
        mode = mode or self.mode
        regions = [(int(lo), int(hi)) for lo, hi in regions]
        self.bytes_moved += sum(hi - lo for p, (lo, hi) in enumerate(regions) if p != self.rank and hi > lo)
        if mode in PEER_MAPPED_MODES and self._win is not None:
            return self._exchange_window(regions, kernel=(mode == "xgmi"))
        if mode in PEER_MAPPED_MODES:
            return self._exchange_ipc(regions, kernel=(mode == "xgmi"), ready=ready, synced=synced,
                                      seq=seq if self._signals is not None else None)
        if mode == "bcast":
            return self._exchange_bcast(regions)
        if mode == "allgather":
            return self._exchange_allgather(regions)
        if mode != "p2p":
            raise ValueError(f"unknown exchange mode {mode!r}")
        import torch.distributed as dist
        lo_me, hi_me = regions[self.rank]
        ops_ = []
        for p in range(self.n_ranks):
            if p == self.rank:
                continue
            if hi_me > lo_me:
                ops_.append(dist.P2POp(dist.isend, self.arena[lo_me:hi_me], self._global_rank(p), self.group))
            lo, hi = regions[p]
            if hi > lo:
                ops_.append(dist.P2POp(dist.irecv, self.arena[lo:hi], self._global_rank(p), self.group))
        if not ops_:
            return []
        return dist.batch_isend_irecv(ops_)

    def _exchange_bcast(self, regions):
        import torch.distributed as dist
        if all(hi <= lo for lo, hi in regions):
            return []
        outs = [self.arena[lo:hi] for lo, hi in regions]
        if self.backend() == "nccl":
            # ProcessGroupNCCL turns an uneven all_gather into one coalesced group of broadcasts.
            return [dist.all_gather(outs, outs[self.rank], group=self.group, async_op=True)]
        works = []
        for r, t in enumerate(outs):
            if t.numel():
                works.append(dist.broadcast(t, src=self._global_rank(r), group=self.group, async_op=True))
        return works

    def _slab_plan(self, regions):
        """Equal-size slab per rank; a region near the arena end starts earlier so the slab stays
        inside the arena (receivers use only [lo, hi) of it)."""
        slab = max(hi - lo for lo, hi in regions)
        n = self.arena.numel()
        return slab, [max(0, min(lo, n - slab)) for lo, _ in regions]

    def _exchange_allgather(self, regions):
        import torch.distributed as dist
        slab, starts = self._slab_plan(regions)
        if slab == 0:
            return []
        if self._gather_bufs is None or self._gather_cap < slab:
            if self._gather_bufs is not None:
                self.sync()  # no unpack still reads the old buffers
            self._gather_cap = max(self._gather_cap, slab)
            self._gather_bufs = [torch.empty(self.n_ranks * self._gather_cap, dtype=torch.uint8, device=self.device)
                                 for _ in range(2)]
            self._gather_used = [False, False]
            if self.is_cuda:
                self._unpack_stream = role_stream(self.device, "unpack")
                self._unpacked = [torch.cuda.Event() for _ in range(2)]
        b = self._gather_n % 2
        self._gather_n += 1
        buf = self._gather_bufs[b][: self.n_ranks * slab]
        if self.is_cuda and self._gather_used[b]:
            # the collective may overwrite this buffer only after its previous use was unpacked
            torch.cuda.current_stream(self.device).wait_event(self._unpacked[b])
        me = starts[self.rank]
        inp = self.arena[me:me + slab]
        if self.backend() == "nccl":
            work = dist.all_gather_into_tensor(buf, inp, group=self.group, async_op=True)
        else:
            work = dist.all_gather(list(buf.view(self.n_ranks, slab).unbind(0)), inp, group=self.group,
                                   async_op=True)

        def unpack():
            for p, (lo, hi) in enumerate(regions):
                if p != self.rank and hi > lo:
                    o = p * slab + lo - starts[p]
                    self.arena[lo:hi].copy_(buf[o:o + hi - lo])

        if not self.is_cuda:
            work.wait()
            unpack()
            return []
        with torch.cuda.stream(self._unpack_stream):
            work.wait()  # the unpack stream waits for the collective, the compute stream does not
            unpack()
            self._unpacked[b].record(self._unpack_stream)
        self._gather_used[b] = True
        return [StreamJoin(self._unpack_stream)]

    def _exchange_ipc(self, regions, kernel: bool = False, ready=None, synced: bool = False, seq=None):
        """Pull every peer's region from its mapped arena: DMA copies (``ipc``) or one K8 gather
        kernel (``xgmi``).  With `seq`, each exchange stream first waits (on the GPU) for the
        counters of the owners it reads."""
        import torch.distributed as dist
        sig = self._signals if seq is not None else None
        if sig is None and not synced:
            if ready is None:  # everything queued so far on this rank
                ready = torch.cuda.Event()
                ready.record(torch.cuda.current_stream(self.device))
            t0 = time.perf_counter()
            ready.synchronize()
            t1 = time.perf_counter()
            dist.barrier(group=self._host_group)
            hw = self.host_wait_s
            hw["event"] += t1 - t0
            hw["barrier"] += time.perf_counter() - t1
            hw["calls"] += 1
        H = ops.hip()
        recv = [(p, lo, hi) for p, (lo, hi) in enumerate(regions) if p != self.rank and hi > lo]
        if kernel:
            segs = [(self._peer_arenas[p].data_ptr() + lo, self.arena.data_ptr() + lo, hi - lo) for p, lo, hi in recv]
            st = self._ipc_streams[0]
            if sig is not None:
                for p, _, _ in recv:
                    sig.wait_on(p, int(seq), st.cuda_stream)
            for i in range(0, len(segs), 16):
                part = segs[i:i + 16]
                H.peer_gather([a for a, _, _ in part], [b for _, b, _ in part], [n for _, _, n in part],
                              st.cuda_stream)
            self._inject_gather_fault(recv, st)
            return [StreamJoin(st)] if segs else []
        used = []
        for i, (p, lo, hi) in enumerate(recv):
            # peers dealt round-robin over the streams (7 peers on 4 streams: 2/2/2/1 copies each;
            # picking by len(used) put peers 5-7 behind peer 1 on the first stream)
            st = self._ipc_streams[i % len(self._ipc_streams)]
            if st not in used:
                used.append(st)
            if sig is not None:
                sig.wait_on(p, int(seq), st.cuda_stream)
            H.memcpy_async(self.arena.data_ptr() + lo, self._peer_arenas[p].data_ptr() + lo, hi - lo, st.cuda_stream)
        if used:
            self._inject_gather_fault(recv, used[-1], used)
        return [StreamJoin(st) for st in used]

    def _inject_gather_fault(self, recv, st, streams=()):
        """ZEST_VMM_FAULT=gather: flip the first 16 bytes of every received region (after the
        copies, on the exchange stream), as a broken peer mapping would."""
        if vmm_fault() != "gather" or not recv:
            return
        for other in streams:
            if other is not st:
                st.wait_stream(other)
        with torch.cuda.stream(st):
            for _, lo, hi in recv:
                v = self.arena[lo:lo + min(16, hi - lo)]
                v.bitwise_not_()

    # -- autotune -----------------------------------------------------------------------------
    def autotune(self, region_lists, modes=EXCHANGE_MODES, passes: int = 2) -> dict:
        """Time each strategy over `region_lists` (a few rounds' regions) and keep the fastest (setup,
        untimed).  Per mode: one pass that also sets up RCCL's connections and buffers, then a timed
        pass.  Timings are MAX-reduced, so every rank picks the same mode.  The arena's contents are
        overwritten (run it before the data lands)."""
        import torch.distributed as dist
        if self.n_ranks == 1:
            return {}
        modes = tuple(m for m in modes if m not in PEER_MAPPED_MODES or self._peer_arenas is not None)
        if self.is_cuda and self.backend() == "gloo":
            # gloo moves device tensors only through its collectives; a batched isend/irecv of
            # device tensors never completed (2-rank rehearsal on one GPU)
            modes = tuple(m for m in modes if m != "p2p")
            if self._peer_arenas is not None:
                # ...and stages them through host memory (device -> host -> TCP -> host -> device):
                # with the arenas peer-mapped, only the modes that move device memory directly are
                # worth timing (the gloo sweep alone took 1.9-4.1 s of a 2-3-rank rehearsal's setup,
                # profiles/r4/swarm_pull_r4r.json, and never won)
                modes = tuple(m for m in modes if m in PEER_MAPPED_MODES)
        # Time on a 256 MiB prefix of every region: bandwidth over xGMI is flat well below a 1 GiB
        # round, and a sweep of full rounds (modes x passes x rounds) cost seconds of setup in the
        # one-GPU rehearsal, where gloo stages device tensors through the host
        # (profiles/r4/swarm_pull_r4b.json).  Much smaller prefixes drown the modes' differences in
        # fixed costs (32 MiB: every mode 0.080 s in a 4-rank rehearsal, profiles/r4/rehearsal_n4_r4c.log).
        cap = int(os.environ.get("ZEST_AUTOTUNE_MB", "256")) << 20
        region_lists = [[(lo, min(hi, lo + cap)) if hi > lo else (lo, hi) for lo, hi in regs] for regs in region_lists]
        times = {}
        moved = self.bytes_moved
        for mode in modes:
            for _ in range(passes):
                self.sync()
                dist.barrier(group=self.group)
                t0 = time.perf_counter()
                try:
                    works = []
                    for regs in region_lists:
                        works += self.exchange(regs, mode)
                    for w in works:
                        w.wait()
                    self.sync()
                    elapsed = time.perf_counter() - t0
                except (RuntimeError, ValueError):  # argument checks fail the same way on every rank
                    elapsed = float("inf")
                dt = torch.tensor([elapsed], dtype=torch.float64, device=self.device if self.is_cuda else "cpu")
                dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=self.group)
                times[mode] = float(dt.item())
        self.bytes_moved = moved
        self.mode = min(modes, key=lambda m: times[m])
        self.times = times
        if self.mode != "allgather":
            self._gather_bufs = None
        _TUNED[(self.n_ranks, self.backend(), self.mapped)] = self.mode
        return times
