"""Intra-node swarm pull: every GPU of a node ends up with every tensor of a repository in its HBM,
while each byte crosses the network (peers / CDN / local xorb cache) exactly once.

    # one process per GPU (torchrun), backend "nccl" = RCCL over xGMI
    tensors = swarm_pull("meta-llama/Llama-3.1-70B")   # collective; every rank gets all tensors
    tensors = zest_amd.pull("meta-llama/Llama-3.1-70B", device="all")   # the same, public API

This is the bench engine's shape (zest_amd.engine.DevicePuller) fed by the network instead of a
pinned synthetic origin:

  plan      rank 0 asks the CAS for every Xet file's reconstruction once; all ranks lay the files out
            in one HBM arena and split the model's *terms* (not whole files) into byte-balanced
            contiguous shares, one per rank, each cut into rounds of ~`round_bytes` (tapered head and
            tail) -- at 8 ranks a 141 GB model is 8 shares of 17.6 GB, whatever the
            shard sizes are (whole-file ownership left 2 of 8 ranks idle in the last of 4 rounds)
  fetch     each rank pulls its round's term ranges device-direct (`_hip.DeviceXetPull.pull_terms`:
            cache -> P2P -> CDN waterfall into pinned staging, GPU LZ4/BG4 decode + BLAKE3 chunk
            hashes straight into the arena and the shared chunk-hash table); CPU process groups use
            the host twin (`_core.HostXetFetcher.fetch_terms`)
  agree     one small all_gather on a gloo control group per round: every rank learns which fetches
            worked and every fetched range's chunk sizes (parsed from the xorb headers)
  exchange  the round's regions are replicated over xGMI by the strategy `RoundExchange.autotune`
            measured fastest at setup (coalesced RCCL broadcasts, slab all-gather, batched p2p, or
            the peer-mapped HIP VMM `ipc` DMA copies / K8 `xgmi` gather kernel), asynchronously:
            round k's exchange overlaps round k+1's fetch
  verify    as each round lands, every receiver BLAKE3-hashes the received chunks itself on a side
            stream; at the end one Merkle launch per rank checks every file against its published
            Xet hash -- no rank trusts another's hashes
  repair    files that fail anywhere are refetched from the CDN by the owners of their terms (their
            peer / cache runs dropped) and re-exchanged over a plain RCCL broadcast
  settle    quarantined peer runs are published to the local xorb cache once their file verified

Elastic re-shard: a fetch that fails on its owner is reassigned to a rank that has not
tried it yet (least queued bytes); an owner that fails twice is dropped from ownership and its queue
moves to the others.  Every rank derives the same plan from the all-gathered round results, so the
collective never diverges; only when no owner is left for a range do all ranks raise SwarmPullError
together.  A rank that *dies* (process exit, hang) is handled by `_Membership`: survivors detect it
through a failed or timed-out control collective plus stale store heartbeats, agree on the survivor
set through the rendezvous store, rebuild their control and data groups without it (in-process, no
exec), and re-shard its unfinished ranges -- ranges some survivor already holds are re-sent from
there, the rest are refetched.

Reference counterpart: python/zest/__init__.py:49-52 (pull) over parallel_download.zig:91-204 (16
concurrent term fetches, batch barrier, ordered writes); the reference has no intra-node swarm, and
its only failure handling is the per-term waterfall (CONTRIBUTING.md:92-99).
"""
from __future__ import annotations

import collections
import json
import os
import threading
import time
import uuid
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from .. import _core, ops
from .. import device as zdev
from .exchange import (_WINDOWS, EXCHANGE_MODES, PEER_MAPPED_MODES, RoundExchange, peer_windows, role_stream,
                       tuned_mode, window_key)
from .split import even_bounds

FILE_ALIGN = 4096
HEAD_TAPER = (0.25, 0.5)
TAIL_TAPER = (0.5, 0.25, 0.125)


def staging_slot_bytes(staging_bytes: int, round_bytes: int, world: int) -> int:
    """Staging slot size of a round-synchronous device swarm pull (`_rounds`: ZEST_SWARM_STREAM=0,
    and the reassigned ranges after a recovery) at `world` ranks.

    There every round is one pull_terms call, and a call drains its pipeline before it returns: with
    1 GiB staging slots a 1 GiB round was a single batch (its H2D and its kernels in series).  Slots
    of a quarter round keep 4 batches in flight within a round: public-path row 81.0 -> 92.4 GB/s at
    2 ranks, 108.6 -> 133.8 at 4 (one shared GPU, 8B random, profiles/r5/swarm_staging_r5as/).
    Round 5 gave 4 and 8 ranks half-round slots because quarter slots "stalled one pull in three";
    that stall was the hash-table zero-fill racing the first ingest kernels (a CDN repair,
    docs/ARCHITECTURE.md 16.2), fixed in _alloc_tables, so every N > 1 takes quarter slots again.
    N = 1 pulls its share in one call and keeps the large slots.  (Streamed pulls size their slots
    in _Swarm.__init__.)
    """
    if world <= 1:
        return int(staging_bytes)
    return min(int(staging_bytes), max(64 << 20, int(round_bytes) // 4))


def _window_shape() -> tuple[int, int]:
    """(slot bytes, slots) of the exchange windows: ZEST_SWARM_WINDOW_MB (256) x ZEST_SWARM_WINDOW_SLOTS
    (4) -- a round's region larger than a slot goes through it in several window rounds."""
    return (max(1, int(os.environ.get("ZEST_SWARM_WINDOW_MB", "256"))) << 20,
            max(2, int(os.environ.get("ZEST_SWARM_WINDOW_SLOTS", "4"))))


class SwarmPullError(RuntimeError):
    pass


@dataclass
class _Agree:
    """One streamed round's pending agreement (see _Swarm._rounds_streamed)."""
    rno: int
    items: list      # item per rank (None: nothing)
    err: str         # this rank's fetch error text ("" = ok)
    info: dict       # this rank's fetch counters
    works: list      # the round's exchange works (the received chunks are hashed after them)
    outs: list       # gathered [status, sizes...] per rank
    work: object     # the async all_gather
    nck: list        # chunks of each rank's item


class _AgreeThread:
    """Finishes a streamed pull's round agreements in order on a thread of its own
    (_Swarm._finish_agree: wait for the round's gather, apply it, hash the received chunks).  The
    first error stops the processing (later rounds are dropped) and is re-raised by raise_error()
    on the pulling thread."""

    def __init__(self, sw: "_Swarm"):
        import queue
        self.sw = sw
        self.q: "queue.Queue" = queue.Queue()
        self.error: BaseException | None = None
        self.abandon = False
        self.busy_s = 0.0
        self.th = threading.Thread(target=self._run, name="zest-swarm-agree", daemon=True)
        self.th.start()

    def _run(self):
        if os.environ.get("ZEST_BENCH_PYPROF") == "1":  # (bench.py: a Python profile of this thread too)
            import cProfile
            import io
            import pstats
            prof = cProfile.Profile()
            prof.enable()
            try:
                self._loop()
            finally:
                prof.disable()
                buf = io.StringIO()
                pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(15)
                import sys
                print(f"[swarm_pull agree thread] Python profile:\n{buf.getvalue()}", file=sys.stderr, flush=True)
            return
        self._loop()

    def _loop(self):
        try:  # (the thread's name in /proc: bench.py's per-thread CPU accounting)
            import ctypes
            ctypes.CDLL(None).prctl(15, b"zest-agree", 0, 0, 0)
        except Exception:  # noqa: BLE001
            pass
        if self.sw.cuda:
            torch.cuda.set_device(self.sw.device)  # (HIP's current device is per thread)
        while True:
            ag = self.q.get()
            if ag is None:
                return
            if self.error is not None or self.abandon:
                continue
            t = time.perf_counter()
            try:
                self.sw._finish_agree(ag)
            except BaseException as e:  # noqa: BLE001 - handed to the pulling thread
                self.error = e
            self.busy_s += time.perf_counter() - t

    def put(self, ag) -> None:
        self.q.put(ag)

    def close(self, abandon: bool = False) -> None:
        """Wait until every queued agreement is finished (abandon: skip those not started)."""
        self.abandon = abandon
        self.q.put(None)
        self.th.join()

    def raise_error(self) -> None:
        if self.error is not None:
            raise self.error


class _RankLost(RuntimeError):
    """A collective failed or timed out: some rank is gone (handled by _Membership.rebuild)."""


# ----------------------------------------------------------------------------------------------
# Planning: byte-balanced contiguous term shares, cut into tapered rounds
# ----------------------------------------------------------------------------------------------
def split_bytes(ulen: np.ndarray, a: int, b: int, weights) -> list[tuple[int, int]]:
    """Cut terms [a, b) into len(weights) contiguous ranges of byte sizes ~ proportional to weights
    (whole terms; empty ranges allowed)."""
    n = len(weights)
    if b <= a:
        return [(a, a)] * n
    cu = np.cumsum(ulen[a:b].astype(np.float64))
    frac = np.cumsum(np.asarray(weights, dtype=np.float64))
    frac /= frac[-1]
    cuts = [a] + [a + int(np.searchsorted(cu, cu[-1] * frac[k], side="left")) + 1 for k in range(n - 1)] + [b]
    cuts = np.maximum.accumulate(np.minimum(np.array(cuts), b))
    return [(int(cuts[k]), int(cuts[k + 1])) for k in range(n)]


def round_weights(share_bytes: int, round_bytes: int, taper: bool = True) -> list[float]:
    """Relative sizes of a share's rounds: full rounds of `round_bytes`, with geometrically shrinking
    first and last rounds (nothing overlaps the first fetch or the last exchange).
    ZEST_SWARM_HEAD_TAPER / ZEST_SWARM_TAIL_TAPER (comma lists of round fractions) override the
    tapers."""
    head = _taper_env("ZEST_SWARM_HEAD_TAPER", HEAD_TAPER)
    tail = _taper_env("ZEST_SWARM_TAIL_TAPER", TAIL_TAPER)
    n = max(1, -(-int(share_bytes) // int(round_bytes)))
    if not taper or n < 4:
        return [1.0] * n
    mid = max(1, -(-int(share_bytes - (sum(head) + sum(tail)) * round_bytes) // round_bytes))
    return list(head) + [1.0] * mid + list(tail)


def _taper_env(name: str, default) -> tuple:
    v = os.environ.get(name, "").strip()
    return tuple(float(x) for x in v.split(",") if x.strip()) if v else tuple(default)


def assign_owners(ulen: np.ndarray, held: np.ndarray | None, world: int) -> np.ndarray:
    """Owner rank of every term.  `held` (bool [world, n_terms], or None) says which rank's local
    xorb cache already covers which term.

    Possession first (the reference's per-term waterfall is cache-first, xet_bridge.zig:161-170):
    consecutive terms held by the same set of ranks are split byte-balanced among those holders,
    least-loaded holder first -- a rank that holds the whole model becomes the node's seeder and its
    peers fetch nothing from the network; a cache shared by every rank is read 1/world per rank.
    The terms nobody holds are then water-filled: cut contiguously (rank order) so that every rank's
    total ends as close to 1/world of the model as the held shares allow.  With nothing held this is
    the plain byte-balanced contiguous split."""
    nt = len(ulen)
    owner = np.full(nt, -1, dtype=np.int64)
    if held is None or not nt or not held.any():
        # nothing held: the plain byte-balanced contiguous split, cut exactly where the bench
        # engine cuts its origin shares (split.even_bounds, integer arithmetic)
        b = even_bounds(ulen, world)
        for r in range(world):
            owner[b[r]:b[r + 1]] = r
        return owner
    load = np.zeros(world, dtype=np.float64)
    u = ulen.astype(np.float64)
    if held is not None and nt and held.any():
        cols = np.ascontiguousarray(held.T.astype(bool))
        change = np.concatenate([[True], (cols[1:] != cols[:-1]).any(axis=1)]) if nt > 1 else np.array([True])
        starts = np.flatnonzero(change).tolist() + [nt]
        for a, b in zip(starts[:-1], starts[1:]):
            who = np.flatnonzero(cols[a])
            if not len(who):
                continue
            order = sorted(who.tolist(), key=lambda r: (load[r], r))
            for (x, y), r in zip(split_bytes(ulen, a, b, [1.0] * len(order)), order):
                owner[x:y] = r
                load[r] += u[x:y].sum()
    free = np.flatnonzero(owner < 0)
    if len(free):
        total = load.sum() + u[free].sum()
        target = np.maximum(total / world - load, 0.0)
        if target.sum() <= 0:
            target = np.ones(world)
        cu = np.cumsum(u[free])
        frac = np.cumsum(target) / target.sum()
        cuts = [0] + [int(np.searchsorted(cu, cu[-1] * frac[k], side="left")) + 1 for k in range(world - 1)] + [len(free)]
        cuts = np.maximum.accumulate(np.minimum(np.array(cuts), len(free)))
        for r in range(world):
            owner[free[cuts[r]:cuts[r + 1]]] = r
    return owner


def rank_items(ulen: np.ndarray, owner: np.ndarray, rank: int, weights) -> list[tuple[int, int]]:
    """`rank`'s terms as contiguous items: its share cut into len(weights) byte-proportional rounds,
    and additionally at every gap between its runs (an item is one contiguous term range)."""
    idx = np.flatnonzero(owner == rank)
    if not len(idx):
        return []
    cu = np.cumsum(ulen[idx].astype(np.float64))
    frac = np.cumsum(np.asarray(weights, dtype=np.float64))
    frac /= frac[-1]
    cut = {int(np.searchsorted(cu, cu[-1] * frac[k], side="left")) + 1 for k in range(len(weights) - 1)}
    gaps = set((np.flatnonzero(np.diff(idx) != 1) + 1).tolist())
    pos = sorted({0} | {p for p in cut | gaps if 0 < p < len(idx)})
    ends = pos[1:] + [len(idx)]
    return [(int(idx[a]), int(idx[b - 1]) + 1) for a, b in zip(pos, ends)]


class _Plan:
    """The repository's Xet files laid out in one arena and their terms as one global table."""

    def __init__(self, files: list[dict], shapes: list[list[tuple[int, int]]]):
        self.files = files
        self.file_off = []
        off = 0
        for f in files:
            self.file_off.append(off)
            off = (off + f["size"] + FILE_ALIGN - 1) // FILE_ALIGN * FILE_ALIGN
        self.arena_bytes = off
        nt = sum(len(s) for s in shapes)
        self.t_file = np.zeros(nt, np.int32)
        self.t_idx = np.zeros(nt, np.int32)       # term index inside its file's reconstruction
        self.t_ulen = np.zeros(nt, np.int64)
        self.t_nck = np.zeros(nt, np.int64)
        self.t_dst = np.zeros(nt, np.int64)       # arena offset of the term's output
        k = 0
        for i, (f, sh) in enumerate(zip(files, shapes)):
            pos = self.file_off[i]
            if sum(u for u, _ in sh) != f["size"]:
                raise SwarmPullError(f"{f['path']}: reconstruction covers {sum(u for u, _ in sh)} bytes, "
                                     f"listing says {f['size']}")
            for j, (u, c) in enumerate(sh):
                self.t_file[k], self.t_idx[k], self.t_ulen[k], self.t_nck[k], self.t_dst[k] = i, j, u, c, pos
                pos += u
                k += 1
        self.t_c0 = np.concatenate([[0], np.cumsum(self.t_nck)[:-1]]).astype(np.int64) if nt else np.zeros(0, np.int64)
        self.n_chunks = int(self.t_nck.sum())
        self.file_t0 = np.searchsorted(self.t_file, np.arange(len(files)), side="left")
        self.file_t1 = np.searchsorted(self.t_file, np.arange(len(files)), side="right")

    def region(self, a: int, b: int) -> tuple[int, int]:
        if b <= a:
            return (0, 0)
        return int(self.t_dst[a]), int(self.t_dst[b - 1] + self.t_ulen[b - 1])

    def jobs(self, a: int, b: int, base_ptr: int) -> list:
        """(xet_hash, t0, t1, dst_ptr, chunk0) per file touched by terms [a, b)."""
        out = []
        t = a
        while t < b:
            f = int(self.t_file[t])
            e = min(b, int(self.file_t1[f]))
            out.append((self.files[f]["xet_hash"], int(self.t_idx[t]), int(self.t_idx[e - 1]) + 1,
                        base_ptr + int(self.t_dst[t]), int(self.t_c0[t])))
            t = e
        return out

    def files_of(self, a: int, b: int) -> list[int]:
        return sorted(set(int(x) for x in self.t_file[a:b])) if b > a else []


class _Deadline:
    """Bounded section: if the block has not finished within `seconds`, the process exits with
    status 3 after a message (and, with faulthandler, every thread's stack).  For the recovery after
    a lost rank: aborting an RCCL communicator, synchronizing the device and building new groups can
    each wait forever on a peer that is gone; a survivor stuck there must fail, not hang the job.
    Exit, never re-exec (a process that initialised the GPU must not replace itself)."""

    def __init__(self, seconds: float, what: str):
        self.seconds, self.what = float(seconds), what
        self._done = threading.Event()
        self._t = None

    def _watch(self):
        if self._done.wait(self.seconds):
            return
        import sys
        print(f"[zest swarm] {self.what} did not finish within {self.seconds:.0f}s "
              f"(ZEST_SWARM_RECOVER_TIMEOUT); exiting", file=sys.stderr, flush=True)
        try:
            import faulthandler
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:  # noqa: BLE001
            pass
        os._exit(3)

    def __enter__(self):
        if self.seconds > 0:
            self._t = threading.Thread(target=self._watch, daemon=True, name="zest-deadline")
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._done.set()
        return False


# ----------------------------------------------------------------------------------------------
# Membership: survivors of a lost rank rebuild their groups in-process
# ----------------------------------------------------------------------------------------------
class _Membership:
    """Who is still in the pull, and the groups they talk over.

    ``ctl`` is a gloo group with a bounded timeout (ZEST_SWARM_CTL_TIMEOUT, default 120 s) carrying
    the per-round agreement; ``data`` carries the piece exchange (RCCL on GPUs).  A heartbeat thread
    stamps ``hb/<global rank>`` in the rendezvous store every second.  When a collective fails or
    times out, `rebuild` posts this rank as alive for the next epoch, waits until every other rank
    has either posted or gone stale (no heartbeat for ZEST_SWARM_HB_STALE s, default 5), lets the first
    survivor publish the member list with a compare-and-set (so all survivors agree), and builds new
    groups over the survivors only (use_local_synchronization: the dead rank takes no part)."""

    def __init__(self, group, backend: str, device: torch.device):
        self.backend = backend
        self.device = device
        self.granks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
        self.me = dist.get_rank()
        self.data = group
        self.timeout_s = float(os.environ.get("ZEST_SWARM_CTL_TIMEOUT", "120"))
        self.stale_s = float(os.environ.get("ZEST_SWARM_HB_STALE", "5"))
        import datetime
        self._td = datetime.timedelta(seconds=self.timeout_s)
        # A control group of our own with a bounded timeout, even over a gloo job: a collective whose
        # peer died must fail in bounded time on EVERY survivor (ranks that wait on a live neighbour
        # that already left the collective would otherwise sit out the job group's 30-minute default).
        # A subgroup's members create it alone (the other ranks of the job are not in this call).
        self.ctl = dist.new_group(ranks=self.granks, backend="gloo", timeout=self._td,
                                  use_local_synchronization=group is not None)
        self._own_data = False
        if backend == "gloo":
            self.data = self.ctl  # CPU (or one-GPU gloo) exchanges: the same bounded timeout
        elif os.environ.get("ZEST_SWARM_ELASTIC", "1") != "0" and len(self.granks) > 1:
            # a data group of our own, so a lost rank's recovery can abort it without touching the
            # caller's group (aborting the default group would leave nothing to rebuild from)
            self.data = dist.new_group(ranks=self.granks, backend=backend, use_local_synchronization=group is not None)
            self._own_data = True
        self.epoch = 0
        self.pulls = 0  # pulls made with this membership (a kept one serves several; store keys per pull)
        self.store = None
        self._stop = threading.Event()
        self._hb = None
        self.enabled = os.environ.get("ZEST_SWARM_ELASTIC", "1") != "0" and "MASTER_ADDR" in os.environ \
            and "MASTER_PORT" in os.environ and len(self.granks) > 1
        tok = [uuid.uuid4().hex if self.rank == 0 else None]
        dist.broadcast_object_list(tok, src=self.granks[0], group=self.ctl)
        self.prefix = f"zest/swarm/{tok[0]}"
        if self.enabled:
            try:
                # store clients of our own, one per thread (a client is not safe to share between
                # threads): the heartbeat thread's, and the main thread's for the membership votes
                def client():
                    return dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), is_master=False,
                                         timeout=self._td)
                self.store = client()
                self._hb_store = client()
                self._beat()
                self._hb = threading.Thread(target=self._heartbeat, daemon=True)
                self._hb.start()
            except Exception:  # noqa: BLE001 - no store: a lost rank fails the pull (no recovery)
                self.enabled = False

    @property
    def rank(self) -> int:
        return self.granks.index(self.me)

    @property
    def world(self) -> int:
        return len(self.granks)

    def _beat(self):
        self._hb_store.set(f"{self.prefix}/hb/{self.me}", repr(time.time()))

    def _heartbeat(self):
        while not self._stop.wait(1.0):
            try:
                self._beat()
            except Exception:  # noqa: BLE001
                return

    def _last_beat(self, g: int) -> float:
        k = f"{self.prefix}/hb/{g}"
        try:
            return float(self.store.get(k)) if self.store.check([k]) else 0.0
        except Exception:  # noqa: BLE001
            return 0.0

    def close(self):
        # stop the heartbeat thread before the caller tears the process down: a daemon thread caught
        # inside a store call at interpreter exit aborted the process (SIGABRT) now and then
        self._stop.set()
        if self._hb is not None:
            self._hb.join(timeout=10)

    def rebuild(self) -> list[int]:
        """Agree on the survivors, rebuild ctl/data groups over them; returns the lost ranks
        (indices into the previous member list)."""
        if not self.enabled:
            raise SwarmPullError("a rank was lost and elastic recovery is off (ZEST_SWARM_ELASTIC=0 or no store)")
        self.epoch += 1
        ek = f"{self.prefix}/e{self.epoch}"
        self.store.set(f"{ek}/alive/{self.me}", "1")
        t_end = time.monotonic() + self.timeout_s + 2 * self.stale_s
        while True:
            now = time.time()
            alive, pending = [], []
            for g in self.granks:
                if self.store.check([f"{ek}/alive/{g}"]):
                    alive.append(g)
                elif now - self._last_beat(g) < self.stale_s:
                    pending.append(g)  # still beating: it is stuck in (or leaving) a collective
            if not pending or time.monotonic() > t_end:
                break
            time.sleep(0.2)
        got = self.store.compare_set(f"{ek}/members", "", json.dumps(sorted(alive)))
        members = json.loads(got)
        if self.me not in members:
            raise SwarmPullError(f"rank {self.me} was dropped from the swarm (epoch {self.epoch})")
        lost = [i for i, g in enumerate(self.granks) if g not in members]
        old_data = self.data
        self.granks = members
        self.ctl = dist.new_group(ranks=members, backend="gloo", timeout=self._td, use_local_synchronization=True)
        if self.backend == "gloo":
            self.data = self.ctl
        else:
            abort = getattr(dist.distributed_c10d, "_abort_process_group", None)
            if abort is not None and old_data is not None and self._own_data:
                try:
                    abort(old_data)  # in-flight RCCL kernels waiting on the dead rank exit
                except Exception:  # noqa: BLE001
                    pass
            self._own_data = True
            self.data = dist.new_group(ranks=members, backend=self.backend, use_local_synchronization=True)
        return lost


# ----------------------------------------------------------------------------------------------
# Fetchers: device-direct (GPU) or host waterfall (CPU), term ranges into the arena
# ----------------------------------------------------------------------------------------------
class _Fetcher:
    def __init__(self, repo, revision, repo_type, device, p2p, peers, tracker, dht, dht_bootstrap, staging_bytes,
                 threads, parent: "_Fetcher | None" = None, slots: int = 0):
        self.args = (repo, revision, repo_type, p2p, list(peers or []), tracker, dht, list(dht_bootstrap or []))
        self.device = device
        self.staging_bytes, self.threads, self.slots = staging_bytes, threads, slots
        # GPU: a second pipeline is a sibling of the first (own streams + staging, the same Xet
        # session, caches, reconstructions and settle book)
        self.parent = parent
        self._impl = None
        self._warm = None
        self._warm_err = None
        self._lock = threading.Lock()  # `impl` is reached from the reconstruction warm-up thread too
        self._serial = None            # CPU: the side thread of submit()

    def prewarm(self) -> None:
        """Build the pipeline (Xet auth, pinned staging, cache scan, swarm) on a side thread, so it
        comes up while rank 0 lists the repository instead of in front of this rank's first fetch
        (the constructor releases the GIL)."""
        if self._impl is not None or self._warm is not None:
            return

        def build():
            try:
                self._make()
            except Exception as e:  # noqa: BLE001 - raised again by `impl`
                self._warm_err = e
        self._warm = threading.Thread(target=build, daemon=True)
        self._warm.start()

    @property
    def impl(self):
        with self._lock:
            if self._warm is not None:
                self._warm.join()
                self._warm = None
                if self._warm_err is not None:
                    e, self._warm_err = self._warm_err, None
                    raise e
            if self._impl is None:
                self._make()
            return self._impl

    def _make(self):
        if self._impl is None:
            repo, revision, repo_type, p2p, peers, tracker, dht, boot = self.args
            if self.device.type == "cuda" and self.parent is not None:
                self._impl = self.parent.impl.sibling(self.staging_bytes, self.slots)
            elif self.device.type == "cuda":
                self._impl = ops.hip().DeviceXetPull(repo, revision, repo_type, p2p, peers, tracker, dht, boot,
                                                     self.device.index or 0, self.staging_bytes, self.threads,
                                                     self.slots)
            else:
                self._impl = _core.HostXetFetcher(repo, revision, repo_type, p2p, peers, tracker, dht, boot,
                                                  self.threads)

    def shapes(self, xet_hash: str):
        return self.impl.term_shapes(xet_hash)

    def keys(self, xet_hash: str):
        return self.impl.term_keys(xet_hash)

    def reset_reconstructions(self) -> None:
        if self._impl is not None and self.parent is None:  # siblings share the parent's
            self._impl.reset_reconstructions()

    def held(self, hexes, starts, ends) -> np.ndarray:
        return np.frombuffer(self.impl.cached_terms(hexes, starts, ends), dtype=np.uint8).astype(bool)

    def fetch(self, jobs, hashes: torch.Tensor, sizes: torch.Tensor | None, repair: bool = False):
        if self.device.type == "cuda":
            return self.impl.pull_terms(jobs, hashes.data_ptr(), sizes.data_ptr() if sizes is not None else 0, repair)
        return self.impl.fetch_terms(jobs, hashes.data_ptr(), repair)

    def order_after(self, event) -> None:
        """GPU pipelines: queue everything from now on behind `event` (a torch.cuda.Event)."""
        if self.device.type == "cuda" and event is not None:
            self.impl.order_after(event.cuda_event)

    # -- streaming submission (the streamed round loop) ----------------------------------------
    def submit(self, jobs, hashes: torch.Tensor, sizes: torch.Tensor | None):
        """Queue one item (a round's term ranges) behind the ones already submitted; returns a
        ticket.  GPU: the persistent pipeline of DeviceXetPull.submit_terms (no drain between
        items); CPU: the host fetches run one item at a time, in order, on a side thread."""
        if self.device.type == "cuda":
            return ("dev", self.impl.submit_terms(jobs, hashes.data_ptr(), sizes.data_ptr() if sizes is not None else 0))
        if self._serial is None:
            from concurrent.futures import ThreadPoolExecutor
            self._serial = ThreadPoolExecutor(max_workers=1, thread_name_prefix="zest-swarm-item")
        impl = self.impl
        return ("host", self._serial.submit(impl.fetch_terms, jobs, hashes.data_ptr(), False))

    def wait(self, ticket):
        """(error text, results, event): blocks until the item's kernels are queued (GPU; `event`
        is a raw hipEvent_t that completes with them) or its host fetch returned (CPU; no event)."""
        kind, t = ticket
        if kind == "dev":
            err, res, ev = self.impl.wait_item(t)
            return err, res, ev
        try:
            return "", t.result(), None
        except Exception as e:  # noqa: BLE001 - reported through the agreement
            return f"{type(e).__name__}: {e}", [], None

    def drain(self, cancel: bool = False) -> None:
        """Wait for every submitted item and forget them (end of a pull).  `cancel`: items whose
        fetches have not finished are abandoned first (an abandoned streamed phase)."""
        if self._impl is not None and hasattr(self._impl, "stream_reset"):
            self._impl.stream_reset(cancel)
        if self._serial is not None:
            self._serial.shutdown(wait=True)
            self._serial = None

    def join(self) -> None:
        """Wait for a prewarm still running (a rank that never fetched)."""
        w = self._warm
        if w is not None:
            w.join()

    def settle(self, xet_hash: str, ok: bool):
        if self._impl is not None:
            self._impl.settle(xet_hash, ok)

    def stats(self) -> dict:
        return json.loads(self._impl.stats_json()) if self._impl is not None else {}

    def timeline(self) -> dict:
        """Device timeline of this pipeline's last pass (ZEST_DEVICE_TIMING=1; {} otherwise)."""
        if self._impl is None or not hasattr(self._impl, "timeline_json"):
            return {}
        return json.loads(self._impl.timeline_json())

    def cache_writer(self) -> dict:
        """Write-behind cache queue counters (GPU pipelines; {} on CPU)."""
        if self._impl is None or not hasattr(self._impl, "cache_writer_json"):
            return {}
        return json.loads(self._impl.cache_writer_json())


# ----------------------------------------------------------------------------------------------
# The pull
# ----------------------------------------------------------------------------------------------
def _fault_spec() -> dict:
    """ZEST_SWARM_FAULT items: "<rank>:<round>" (that fetch raises), "exit:<rank>:<round>" (that
    rank's process exits at that round; round -1: while the listing / plan is made)."""
    out = {"fail": set(), "exit": set()}
    for item in os.environ.get("ZEST_SWARM_FAULT", "").split(","):
        p = item.split(":")
        if len(p) == 2:
            out["fail"].add((int(p[0]), int(p[1])))
        elif len(p) == 3 and p[0] == "exit":
            out["exit"].add((int(p[1]), int(p[2])))
    return out


class _Swarm:
    def __init__(self, repo, revision, group, device, *, p2p, peers, tracker, dht, dht_bootstrap, repo_type,
                 verify_received, staging_bytes, threads, round_bytes, exchange, reuse=False, possession=True):
        self.t0 = time.perf_counter()
        self.times: dict = {}
        self.repo, self.revision, self.repo_type = repo, revision, repo_type
        backend = str(dist.get_backend(group)).lower()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.backend = backend
        t_m = time.perf_counter()
        # reuse_pipeline pulls also keep their membership (control group, data group, store clients,
        # heartbeat) for the next pull over the same group, unless a rank was lost under it
        self.member_key = (tuple(dist.get_process_group_ranks(group)) if group is not None
                           else tuple(range(dist.get_world_size())), backend, str(self.device))
        kept_m = _MEMBERS.pop(self.member_key, None) if reuse else None
        self.m = kept_m if kept_m is not None and kept_m.epoch == 0 else _Membership(group, backend, self.device)
        if kept_m is not None and kept_m is not self.m:
            kept_m.close()
        self.m.pulls += 1
        self._mark("membership_s", t_m)
        self.verify = verify_received
        self.round_bytes = int(round_bytes)
        self.exchange_req = exchange
        # Streamed rounds (ZEST_SWARM_STREAM, default on at N > 1, _rounds_streamed): one persistent
        # fetch pipeline streams this rank's whole share; exchanges are ordered on the device and the
        # agreement lags.  Its staging: 4 slots of half a round, two rounds buffered ahead of the copy
        # engine.  ZEST_SWARM_STREAM=0 keeps the round-synchronous loop (below), which the streamed
        # phase also falls back to for reassigned ranges.
        self.streamed = os.environ.get("ZEST_SWARM_STREAM", "1") != "0" and self.m.world > 1
        # Cross-round fetch pipelining of the synchronous loop (ZEST_SWARM_PIPELINE, default on at
        # N > 1 when not streamed): round k + 1's ranges are fetched on a second pipeline while round
        # k's fetch drains and is agreed.  On GPUs the second pipeline is a sibling of the first (half
        # the staging, the same Xet session, caches and reconstructions); on CPU groups it is a second
        # host fetcher that joins no DHT (one node per process is enough).
        self.pipelined = (os.environ.get("ZEST_SWARM_PIPELINE", "1") != "0" and self.m.world > 1
                          and not self.streamed)
        slots = int(os.environ.get("ZEST_SWARM_SLOTS", "4")) if self.streamed else 0
        if self.cuda and not os.environ.get("ZEST_SWARM_STAGING_MB"):
            if self.streamed:
                staging_bytes = min(int(staging_bytes), max(64 << 20, self.round_bytes // 2))
            else:
                staging_bytes = staging_slot_bytes(staging_bytes, self.round_bytes, self.m.world)
        self.reuse_key = (repo, revision, repo_type, str(self.device), bool(p2p), tuple(peers or []), tracker,
                          bool(dht), tuple(dht_bootstrap or []), int(staging_bytes), int(threads), self.pipelined,
                          self.streamed, slots, os.environ.get("HF_ENDPOINT"), os.environ.get("ZEST_CACHE_DIR"))
        self.reuse = reuse
        kept = _PIPELINES.pop(self.reuse_key, None) if reuse else None
        self.reused = kept is not None
        self.stats_base: dict = {}
        if kept is not None:  # a previous pull's pipelines: staging pinned, session up; reconstructions anew
            self.fetchers = kept
            self.fetcher = kept[0]
            for f in kept:
                f.reset_reconstructions()
            # the session's counters run on across pulls: this pull reports its own share
            self.stats_base = _merged_stats([f.stats() for f in kept if f.parent is None])
        else:
            self.fetcher = _Fetcher(repo, revision, repo_type, self.device, p2p, peers, tracker, dht, dht_bootstrap,
                                    staging_bytes, threads, slots=slots)
            self.fetcher.prewarm()
            self.fetchers = [self.fetcher]
            if self.pipelined:
                if self.cuda:
                    f2 = _Fetcher(repo, revision, repo_type, self.device, p2p, peers, tracker, False, dht_bootstrap,
                                  max(64 << 20, staging_bytes // 2), threads, parent=self.fetcher, slots=2)
                else:
                    f2 = _Fetcher(repo, revision, repo_type, self.device, p2p, peers, tracker, False, dht_bootstrap,
                                  staging_bytes, threads)
                    f2.prewarm()
                self.fetchers.append(f2)
        self._fut = None
        self.fault = _fault_spec()
        self.possession = possession
        self.stats = {"reassigned": 0, "recovered_ranks": 0, "resent_bytes": 0, "repaired_files": 0,
                      "from_peer": 0, "from_cdn": 0, "from_cache": 0, "fetched_wire_bytes": 0}

    def _mark(self, name, t):
        self.times[name] = round(self.times.get(name, 0.0) + time.perf_counter() - t, 4)

    # -- control plane ------------------------------------------------------------------------
    def _gather(self, obj):
        out = [None] * self.m.world
        try:
            dist.all_gather_object(out, obj, group=self.m.ctl)
        except Exception as e:  # noqa: BLE001 - gloo reports a dead or stuck peer as a RuntimeError
            raise _RankLost(str(e)) from e
        return out

    def _bcast_from0(self, obj):
        box = [obj]
        try:
            dist.broadcast_object_list(box, src=self.m.granks[0], group=self.m.ctl)
        except Exception as e:  # noqa: BLE001
            raise _RankLost(str(e)) from e
        return box[0]

    def _plan_from0(self, obj):
        """Rank 0's listing/plan to every rank.  Through the rendezvous store when there is one: the
        listing (a CAS reconstruction per file) may take longer than the control group's bounded
        timeout on a slow network, so the other ranks wait for as long as rank 0's heartbeat stays
        fresh instead of failing a timed-out collective and rebuilding groups around a rank that is
        only slow.  Without a store: a broadcast on the control group."""
        m = self.m
        if not m.enabled:
            return self._bcast_from0(obj)
        key = f"{m.prefix}/e{m.epoch}/p{m.pulls}/plan"
        if m.rank == 0:
            m.store.set(key, json.dumps(obj))
            return obj
        root, t0 = m.granks[0], time.time()
        while not m.store.check([key]):
            # (a root that has not stamped its first heartbeat yet counts from when this wait began)
            if time.time() - max(m._last_beat(root), t0) > m.stale_s:
                raise _RankLost(f"rank {root} stopped while listing {self.repo}")  # survivors re-plan
            # 2 ms polls for the first second (a plan is usually ready in tens of ms; a fixed 50 ms
            # poll left the other ranks up to 50 ms behind rank 0, which then waited for them in the
            # possession gather: 44 ms of a 0.44 s 2-rank pull, profiles/r5/rehearsal_n2_r5t/lag2.log)
            time.sleep(0.002 if time.time() - t0 < 1.0 else 0.05)
        return json.loads(m.store.get(key))

    # -- setup --------------------------------------------------------------------------------
    def listing_and_plan(self):
        t = time.perf_counter()
        obj = None
        if (self.m.me, -1) in self.fault["exit"]:
            os._exit(1)  # fault injection (tests): this rank dies while the plan is being made
        if self.m.rank == 0:
            try:
                t_l = time.perf_counter()
                commit, files = _core.list_repo_files(self.repo, self.revision, self.repo_type)
                self._mark("plan_list_s", t_l)
                st = [f for f in files if f["path"].endswith(".safetensors")]
                xet = [f for f in st if f["xet_hash"]]
                t_r = time.perf_counter()
                impl = self.fetcher.impl  # (waits for a pipeline still being built)
                self._mark("plan_pipeline_wait_s", t_r)
                t_r = time.perf_counter()
                shapes = _parallel_map(lambda f: [tuple(x) for x in impl.term_shapes(f["xet_hash"])], xet,
                                        max(8, self.fetcher.threads))
                # (xorb hex, chunk range) per term: every rank checks its own cache against them
                keys = [[list(k) for k in impl.term_keys(f["xet_hash"])] for f in xet] if self.possession else None
                self._mark("plan_recon_s", t_r)
                obj = ("ok", commit, st, shapes, keys)
            except Exception as e:  # noqa: BLE001 - every rank leaves the same way
                obj = ("err", f"{type(e).__name__}: {e}")
        t_b = time.perf_counter()
        obj = self._plan_from0(obj)
        self._mark("plan_share_s", t_b)
        if obj[0] != "ok":
            raise SwarmPullError(f"listing/planning {self.repo}@{self.revision} failed on rank 0: {obj[1]}")
        _, self.commit, st_files, shapes, keys = obj
        self.xet_files = [f for f in st_files if f["xet_hash"]]
        self.plain_files = [f for f in st_files if not f["xet_hash"]]
        self.plan = _Plan(self.xet_files, shapes)
        self.term_keys = [k for fk in keys for k in fk] if keys is not None else None
        self._mark("plan_s", t)

    def gather_possession(self):
        """Which terms each rank's xorb cache already covers (have-map): checked
        locally against the planned terms' chunk ranges, then all-gathered as bitmaps on the control
        group.  Sets self.held (bool [world, n_terms]) or None when nobody holds anything.
        The same all-gather carries what allocate() and setup_exchange() need agreed -- whether every
        rank can reuse its kept arena, and the state of its ready-counter page -- so a repeated pull
        pays one control collective here instead of three."""
        self.held = None
        t = time.perf_counter()
        self._arena_local()
        bits = None
        if self.term_keys is not None and len(self.term_keys):
            hexes = [k[0] for k in self.term_keys]
            mine = self.fetcher.held(hexes, [int(k[1]) for k in self.term_keys], [int(k[2]) for k in self.term_keys])
            bits = np.packbits(mine).tobytes()
        mine_v = (bits, self._have_local, self._sig_local[0], self._sig_local[1])
        allv = self._gather(mine_v) if self.m.world > 1 else [mine_v]
        self._have_all = int(all(v[1] for v in allv))
        self._sig_agreed = (bool(all(v[2] for v in allv)), max(int(v[3]) for v in allv))
        if bits is not None:
            nt = len(self.term_keys)
            held = np.stack([np.unpackbits(np.frombuffer(v[0], dtype=np.uint8))[:nt].astype(bool) for v in allv])
            self.held = held if held.any() else None
        self._mark("possession_s", t)

    def _arena_local(self):
        """This rank's side of the arena-reuse and exchange-window decisions (agreed in
        gather_possession)."""
        n = max(1, self.plan.arena_bytes)
        self._want_map = (self.cuda and self.m.world > 1 and os.environ.get("ZEST_EXCHANGE_IPC", "1") != "0"
                          and self.exchange_req in ("auto", "ipc", "xgmi"))
        # reuse_arena True: the arena of this process's previous pull over the same group is reused
        # (bench.py's repeated pulls); None / False (default): a fresh ordinary allocation, freed with
        # the caller's tensors -- the peer-mapped exchanges go through the group's exchange windows
        # (mapped once per process), not through a peer mapping of the arena.
        self._use_cache = self.reuse_arena is True
        self._arena_key = (self.device.index if self.cuda else -1, self.m.world, tuple(self.m.granks))
        cached = _ARENAS.get(self._arena_key) if self._use_cache else None
        self._cached = cached
        self._have_local = int(cached is not None and cached[0].numel() >= n)
        # exchange windows: every rank must already hold the group's windows (of the wanted shape)
        # with a live counter page to use them without a collective; their window-round counts are
        # agreed (max) with the same all-gather
        pw = _WINDOWS.get(window_key(self.device, self.m.data, self.m.world)) if self._want_map else None
        slot, slots = _window_shape()
        self._win_local = (bool(pw is not None and pw.signals is not None and pw.slot_bytes == slot and pw.slots == slots),
                           int(pw.sent) if pw is not None else 0)
        self._sig_local = self._win_local  # (gathered with the possession bits)

    def allocate(self):
        t = time.perf_counter()
        P = self.plan
        n = max(1, P.arena_bytes)
        if not hasattr(self, "_have_all"):  # (no possession gather ran: agree on the arena here)
            self._arena_local()
            allv = self._gather((self._have_local, *self._win_local)) if self.m.world > 1 else \
                [(self._have_local, *self._win_local)]
            self._have_all = int(all(v[0] for v in allv))
            self._sig_agreed = (bool(all(v[1] for v in allv)), max(int(v[2]) for v in allv))
        self.arena = None
        # (device memory free before the arena, and the arena's own allocation time: a pull after
        # another pull in the same process spent 4.5 s here, profiles/r5/bench70b_r5ai.log)
        self.alloc_info = {"free_before_GB": round(torch.cuda.mem_get_info(self.device)[0] / 1e9, 2)} if self.cuda else {}
        t_a = time.perf_counter()
        # reuse_arena=True: the arena of this process's previous pull of at least this size, when
        # every rank has one (a fresh 141 GB arena per pull costs the driver's reclaim of the last
        # one, ~4 s, profiles/r5/alloc_probe_141g_r5aj.log)
        key, use_cache, cached = self._arena_key, self._use_cache, self._cached
        have = self._have_all if use_cache else 0
        self.reused_arena = bool(have)
        self.mapped = None
        if have:
            full = cached[0]
            self.arena = full[:n]
            self.alloc_info["reused"] = True
            self.alloc_info["arena_s"] = round(time.perf_counter() - t_a, 4)
            self._alloc_tables(P)
            self._mark("alloc_s", t)
            return
        _ARENAS.pop(key, None)  # (a smaller cached arena is dropped before the new one is made)
        self.arena = ops.padded_empty(n, self.device) if self.cuda else torch.empty(n + ops.PAD, dtype=torch.uint8)[:n]
        self.alloc_info["arena_s"] = round(time.perf_counter() - t_a, 4)
        self._alloc_tables(P)
        if use_cache:
            _ARENAS[key] = (self.arena, None, _storage_refs(self.arena))
        self._mark("alloc_s", t)

    def _alloc_tables(self, P):
        nck = max(1, P.n_chunks)
        if self.cuda and os.environ.get("ZEST_SWARM_FAULT_SLOWZERO"):
            # fault injection (tests): the current stream is busy for a while, so the zero-fill below
            # runs late -- a pipeline not ordered after it would write chunk hashes that get zeroed
            torch.cuda._sleep(int(os.environ["ZEST_SWARM_FAULT_SLOWZERO"]))
        self.hashes = torch.zeros((nck, 32), dtype=torch.uint8, device=self.device)
        self.sizes = torch.zeros(nck, dtype=torch.int64, device=self.device) if self.cuda else None
        self.lens = np.zeros(nck, dtype=np.uint32)   # every chunk's size, filled as rounds are agreed
        if self.cuda and os.environ.get("ZEST_SWARM_UNORDERED_TABLES") != "1":
            # The fetch pipelines write these tables (and the arena) from streams of their own
            # (DeviceXetPull's compute stream), which are not ordered after torch's current stream:
            # the zero-fill must have run before the first ingest kernel, or it wipes the chunk hashes
            # that kernel wrote and the file fails its Merkle check -> a ~2.5 s CDN repair.  That race
            # was round 5's unexplained 2.4-3.4 s stall: it showed whenever the device ran the two
            # streams concurrently (other staging sizes, other rank counts; at will with 16 hardware
            # queues per process, profiles/r6/), and tests/test_gpu_device.py pins it with a delayed
            # zero-fill (ZEST_SWARM_FAULT_SLOWZERO; ZEST_SWARM_UNORDERED_TABLES=1 brings the race back for
            # that test's negative control).  The pipelines wait for this event on the GPU (_Fetcher.
            # order_after) -- a host synchronize here cost up to 22 ms on a GPU shared by 4 ranks.
            self.tables_ready = torch.cuda.Event()
            self.tables_ready.record(torch.cuda.current_stream(self.device))

    def shard(self):
        """Per-rank queues of items (term ranges), identical on every rank."""
        P = self.plan
        W = self.m.world
        held = getattr(self, "held", None)
        self.owner = assign_owners(P.t_ulen, held, W)
        shares = [int(P.t_ulen[self.owner == r].sum()) for r in range(W)]
        max_share = max(shares, default=0)
        taper = os.environ.get("ZEST_ROUND_TAPER", "1") != "0"
        # One rank: nothing to overlap a fetch with, so the whole share is one pull_terms call (every
        # round boundary drains the fetch pipeline: 16 rounds of 1 GiB cost ~25 ms each on
        # Llama-3.1-8B, profiles/r4/swarm_pull_r4b.json).
        rb = self.round_bytes
        if self.streamed and max_share:
            # streamed rounds cost no drain and no blocking agreement, so the share is cut finer: at
            # least ZEST_SWARM_MIN_ROUNDS (8) rounds per rank (>= 64 MiB each), so the first exchange
            # starts early and the last one is short (8 ranks of an 8B model: 2 GB shares were 2
            # rounds of 1 GiB, the first exchange waiting ~0.3 s, profiles/r6/)
            k = max(1, int(os.environ.get("ZEST_SWARM_MIN_ROUNDS", "8")))
            rb = min(rb, max(64 << 20, -(-max_share // k)))
        self.round_bytes_used = rb
        weights = round_weights(max_share, rb, taper) if max_share and W > 1 else [1.0]
        self.items: list[tuple[int, int]] = []
        self.queue: list[list[int]] = [[] for _ in range(W)]
        for r in range(W):
            for ra, rb in rank_items(P.t_ulen, self.owner, r, weights):
                self.items.append((ra, rb))
                self.queue[r].append(len(self.items) - 1)
        self.held_bytes = [int(P.t_ulen[(self.owner == r) & held[r]].sum()) if held is not None else 0
                           for r in range(W)]
        self.share_bytes = shares
        self.n_rounds_planned = len(weights)
        # Rank 0 holds every reconstruction from planning; the others fetch theirs now, on a side
        # thread, while the arena is mapped and the exchange autotuned, instead of in front of
        # their first fetch.
        self._recon_warm = None
        if self.m.rank != 0 and self.queue[self.m.rank]:
            mine = sorted({f for it in self.queue[self.m.rank] for f in P.files_of(*self.items[it])})
            hexes = [self.xet_files[f]["xet_hash"] for f in mine]

            def warm():
                try:
                    _parallel_map(self.fetcher.shapes, hexes, max(8, self.fetcher.threads))
                except Exception:  # noqa: BLE001 - the fetch itself reports any real failure
                    pass
            self._recon_warm = threading.Thread(target=warm, daemon=True)
            self._recon_warm.start()
        self.tried: dict = {}        # item -> members (global ranks) that failed it
        self.fails: dict = {}        # global rank -> failed fetches
        self.owner_of: dict = {}     # item -> global rank that fetched it
        self.have: set = set()       # items this rank holds (fetched, or received and hashed)
        self.item_lens: dict = {}    # item -> uint32 chunk sizes (bytes), known to every rank
        self.fetched_bytes = 0       # unpacked bytes this rank fetched from the network

    # -- exchange -----------------------------------------------------------------------------
    def setup_exchange(self):
        t = time.perf_counter()
        W = self.m.world
        self.xchg = RoundExchange(self.arena, self.m.rank, W, self.m.data, "p2p")
        if getattr(self, "_want_map", False) and self.m.world > 1:
            # peer-mapped exchanges go through the group's exchange windows: mapped once per process
            # (every rank kept usable ones: no collective, counters continue from the agreed count),
            # else made now (collective); none -> RCCL exchanges only
            t_w = time.perf_counter()
            key = window_key(self.device, self.m.data, self.m.world)
            slot, slots = _window_shape()
            agreed = getattr(self, "_sig_agreed", (False, 0))
            pw = _WINDOWS.get(key) if agreed[0] else peer_windows(self.device, self.m.rank, self.m.world, self.m.data,
                                                                  slot, slots)
            if pw is not None:
                self.xchg.enable_window(pw, resync=agreed[1] if agreed[0] else None)
            self._mark("windows_s", t_w)
        self.verify_stream = role_stream(self.device, "verify") if self.cuda else None
        self._hash_scratch = ops.HashScratch(self.device) if self.cuda else None
        if W == 1:
            self.xchg.mode = "none"
            return
        req = self.exchange_req
        if req != "auto":
            if req in PEER_MAPPED_MODES and not self.xchg.mapped:
                raise SwarmPullError(f"exchange={req}: mapping the peers' arenas failed")
            self.xchg.mode = req
            return
        cached = tuned_mode(W, self.backend, self.xchg.mapped)
        if cached is not None:
            self.xchg.mode = cached
            return
        if not self.cuda:
            self.xchg.mode = "bcast"  # CPU groups: nothing to tune over xGMI
            return
        # time the strategies on the first rounds' planned regions (the arena holds nothing yet)
        regs = []
        for k in range(min(3, max(len(q) for q in self.queue))):
            regs.append([self.plan.region(*self.items[q[k]]) if k < len(q) else (0, 0) for q in self.queue])
        try:
            self.xchg.autotune(regs, EXCHANGE_MODES)
        except Exception as e:  # noqa: BLE001
            raise _RankLost(str(e)) from e
        self._mark("autotune_s", t)

    def _hash_received(self, recv_items, works):
        """Hash the chunks of `recv_items` (owned by peers) once `works` landed; returns an event
        (GPU) marking completion, or None (CPU: done on return)."""
        P = self.plan
        if not self.cuda:
            for w in works:
                w.wait()
            if self.verify:
                for it in recv_items:
                    offs, lens, c0 = self._chunk_layout(it)
                    self.hashes[c0:c0 + len(lens)] = ops.hash_ranges(self.arena, offs, lens)
            self.have.update(recv_items)
            return None
        H = ops.hip()
        # The chunk tables go up first, from pinned memory on the (idle) current stream: a pageable
        # copy issued on the verify stream would block the host until that stream -- which waits for
        # this round's exchange -- got there, serializing the next round's fetch behind the exchange.
        # Every chunk has its own slot in the pull's layout buffers (pinned + device, kept across
        # pulls), so nothing is allocated or pinned per item (a pinned allocation per item and table
        # doubled the pulling process's CPU time in the 8-rank rehearsal).
        jobs = []
        if self.verify:
            up = torch.cuda.current_stream(self.device)
            h_off, h_len, d_off, d_len = _layout_bufs(self.device, max(1, self.plan.n_chunks))
            for it in recv_items:
                offs, lens, c0 = self._chunk_layout(it)
                n = len(lens)
                if not n:
                    continue
                h_off[c0:c0 + n].numpy()[:] = offs.view(np.int64)
                h_len[c0:c0 + n].numpy()[:] = lens.view(np.int32)
                d_off[c0:c0 + n].copy_(h_off[c0:c0 + n], non_blocking=True)
                d_len[c0:c0 + n].copy_(h_len[c0:c0 + n], non_blocking=True)
                jobs.append((d_off[c0:c0 + n], d_len[c0:c0 + n], lens, c0))
            self.verify_stream.wait_stream(up)
        with torch.cuda.stream(self.verify_stream):
            for w in works:
                w.wait()
            for od, ld, lens, c0 in jobs:
                sp, sb = self._hash_scratch.get(len(lens), int(lens.sum(dtype=np.uint64)))
                H.hash_ranges(self.arena.data_ptr(), od.data_ptr(), ld.data_ptr(), len(lens),
                              self.hashes.data_ptr() + 32 * c0, ops.KEY_DATA, self.verify_stream.cuda_stream, sp, sb)
            ev = torch.cuda.Event()
            ev.record(self.verify_stream)
        del P
        return ev

    def _chunk_layout(self, it: int):
        """Arena offsets (uint64), sizes (uint32) and first global chunk of item it's chunks."""
        P = self.plan
        a, b = self.items[it]
        lens = np.frombuffer(self.item_lens[it], dtype=np.uint32)
        nck = P.t_nck[a:b]
        term_of = np.repeat(np.arange(a, b), nck)
        cs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))])
        first = np.concatenate([[0], np.cumsum(nck)[:-1]]).astype(np.int64)  # chunk position of each term
        start_in_term = cs[:-1] - cs[first][np.repeat(np.arange(b - a), nck)]
        offs = (P.t_dst[term_of].astype(np.uint64) + start_in_term).astype(np.uint64)
        return offs, lens, int(P.t_c0[a])

    def _apply_meta(self, meta, info: dict):
        """Apply one round's agreement -- every rank's (item, error text, chunk sizes) -- on this
        rank (every rank derives the same result): a failed item is reassigned to a rank that has
        not tried it (least queued bytes), a rank failing twice hands its queue to the others; the
        rest is recorded (owner, chunk sizes, this rank's fetch counters from `info`).  Returns
        (fatal errors, the round's regions per rank with failed ones empty, items to receive)."""
        P = self.plan
        me = self.m.rank
        fatal, regions, recv = [], [], []
        for r, (item, e, ls) in enumerate(meta):
            if item is None:
                regions.append((0, 0))
                continue
            g = self.m.granks[r]
            if e:
                if not getattr(self, "first_fetch_error", None):
                    self.first_fetch_error = e  # (named in the final error if the item finds no owner)
                self.fails[g] = self.fails.get(g, 0) + 1
                self.tried.setdefault(item, set()).add(g)
                moves = [item]
                if self.fails[g] >= 2:   # a repeatedly failing owner: hand its queue to the others
                    moves += self.queue[r]
                    self.queue[r] = []
                for mv in moves:
                    cands = [q for q in range(self.m.world)
                             if self.fails.get(self.m.granks[q], 0) < 2 and self.m.granks[q] not in self.tried.get(mv, set())]
                    if not cands:
                        fatal.append(e if mv == item else f"no owner left for terms {self.items[mv]} "
                                                          f"(rank {g} dropped; first fetch error: "
                                                          f"{self.first_fetch_error})")
                        continue
                    load = [sum(int(P.t_ulen[self.items[x][0]:self.items[x][1]].sum()) for x in self.queue[q])
                            for q in range(self.m.world)]
                    q = min(cands, key=lambda q: (load[q], q))
                    self.queue[q].append(mv)
                    self.stats["reassigned"] += 1
                regions.append((0, 0))
                continue
            self.item_lens[item] = ls
            first_time = item not in self.owner_of
            self.owner_of.setdefault(item, g)
            regions.append(P.region(*self.items[item]))
            if r == me:
                if first_time and info:
                    a, b = self.items[item]
                    self.fetched_bytes += int(P.t_ulen[a:b].sum())
                    self.stats["fetched_wire_bytes"] += info["fetched"]
                    for k in ("from_peer", "from_cdn", "from_cache"):
                        self.stats[k] += info[k]
                self.have.add(item)
            elif item not in self.have:  # (a re-send also reaches ranks holding it: same bytes)
                recv.append(item)
            if not first_time and r == me:
                a, b = self.items[item]
                self.stats["resent_bytes"] += int(P.t_ulen[a:b].sum())
        return fatal, regions, recv

    # -- streamed rounds (N > 1) ----------------------------------------------------------------
    def _rounds_streamed(self):
        """The engine's shape on the public path, N > 1:

          * every round's item of this rank is submitted up front to ONE persistent fetch pipeline
            (_Fetcher.submit -> DeviceXetPull.submit_terms), which streams them with no drain
            between rounds;
          * round k's exchange is issued as soon as this rank's item k is queued on the GPU and is
            ordered after it on the device -- the owners' ready counters for the peer-mapped modes
            (hipStreamWaitValue32), a stream wait on the item's event for RCCL.  The schedule is
            fixed at planning, so nothing has to be agreed first;
          * the agreement (a status word + the item's chunk sizes) is an asynchronous gloo
            all_gather of one small tensor per rank, waited for only when more than
            ZEST_SWARM_AGREE_LAG (default 3) rounds are pending; a round's received chunks are
            hashed once their sizes are agreed.

        A range whose fetch failed is exchanged anyway (its bytes are never hashed, so never
        trusted) and is reassigned exactly as in the synchronous loop; run() then re-fetches and
        re-sends the reassigned ranges with _rounds()."""
        P = self.plan
        me = self.m.rank
        rounds = []
        while any(self.queue):
            rounds.append(self._pop_round())
        self.unagreed = [list(x) for x in rounds]   # popped, not agreed (re-queued by _recover)
        self.item_ready_s = []  # per round: seconds into the pull when this rank's item was queued
        base = self.arena.data_ptr()
        tickets, injected = [None] * len(rounds), set()
        for k, items in enumerate(rounds):
            it = items[me]
            if it is None:
                continue
            if (self.m.me, self.round_no + k) in self.fault["fail"]:
                injected.add(k)  # fault injection (tests): this fetch "fails"
                continue
            a, b = self.items[it]
            tickets[k] = self.fetcher.submit(P.jobs(a, b, base), self.hashes, self.sizes)
        self._tickets = tickets
        if self.cuda and self.xchg.mode in PEER_MAPPED_MODES:
            # peer-mapped exchanges write this arena from the exchange streams, which wait only for
            # the owners' counters: order them after whatever the caller queued on the arena
            self.xchg.order_after(torch.cuda.current_stream(self.device))
        lag = max(0, int(os.environ.get("ZEST_SWARM_AGREE_LAG", "3")))
        pending = collections.deque()
        # The agreements are finished on a thread of their own (ZEST_SWARM_AGREE_THREAD, default on):
        # a round's received chunks are hashed as soon as its gather completes, instead of when this
        # thread next comes back from waiting for its own item -- and this thread never blocks on a
        # slower peer before its last exchange is issued.
        agree = _AgreeThread(self) if os.environ.get("ZEST_SWARM_AGREE_THREAD", "1") != "0" else None
        try:
            self._stream_loop(rounds, tickets, injected, pending, lag, agree)
        except BaseException:
            if agree is not None:
                agree.close(abandon=True)  # (the rounds not agreed yet stay in self.unagreed)
            raise
        if agree is not None:
            t = time.perf_counter()
            agree.close()
            self._mark("agree_s", t)
            self.times["agree_thread_s"] = round(self.times.get("agree_thread_s", 0.0) + agree.busy_s, 4)
            agree.raise_error()
        self._tickets = []

    def _stream_loop(self, rounds, tickets, injected, pending, lag, agree):
        P = self.plan
        me = self.m.rank
        for k, items in enumerate(rounds):
            rno = self.round_no
            if (self.m.me, rno) in self.fault["exit"]:
                os._exit(1)  # fault injection: this rank dies mid-pull (tests)
            it = items[me]
            t = time.perf_counter()
            err, lens, info, ev = "", b"", {}, None
            if it is not None:
                if k in injected:
                    err = f"rank {self.m.me}: RuntimeError: injected fetch failure (round {rno})"
                else:
                    e, res, ev = self.fetcher.wait(tickets[k])
                    tickets[k] = None
                    if e:
                        err = f"rank {self.m.me}: {e}"
                    else:
                        lens = b"".join(r["chunk_lens"] for r in res)
                        info = {x: sum(r[x] for r in res) for x in ("fetched", "from_peer", "from_cdn", "from_cache")}
            self._mark("fetch_s", t)
            t = time.perf_counter()
            self.item_ready_s.append(round(t - getattr(self, "t_pull", t), 4))
            regions = [P.region(*self.items[x]) if x is not None else (0, 0) for x in items]
            works = []
            if any(hi > lo for lo, hi in regions):
                try:
                    works = self.xchg.exchange_after(regions, ev)
                except Exception as e:  # noqa: BLE001
                    raise _RankLost(str(e)) from e
            self._mark("exchange_issue_s", t)
            ag = self._post_agree(rno, items, err, lens, info, works)
            self.round_no += 1
            if agree is not None:
                agree.put(ag)
                agree.raise_error()  # (a failed agreement: stop issuing; run() recovers or fails)
                continue
            pending.append(ag)
            t = time.perf_counter()
            while pending and (len(pending) > lag or pending[0].work.is_completed()):
                self._finish_agree(pending.popleft())
            self._mark("agree_s", t)
        t = time.perf_counter()
        while pending:
            self._finish_agree(pending.popleft())
        self._mark("agree_s", t)

    def _post_agree(self, rno: int, items: list, err: str, lens: bytes, info: dict, works: list) -> "_Agree":
        """Start round rno's agreement: an async all_gather of [status, chunk sizes...] per rank
        (status 0 ok, 1 failed, 2 nothing to fetch), padded to the round's largest item."""
        P = self.plan
        me = self.m.rank
        nck = [int(P.t_nck[self.items[x][0]:self.items[x][1]].sum()) if x is not None else 0 for x in items]
        mine = torch.zeros(1 + max(nck), dtype=torch.int32)
        if items[me] is None:
            mine[0] = 2
        elif not err:
            arr = np.frombuffer(lens, dtype=np.int32)
            if len(arr) != nck[me]:
                err = f"rank {self.m.me}: {len(arr)} chunk sizes for a range of {nck[me]} chunks"
            else:
                mine[1:1 + len(arr)] = torch.from_numpy(arr.copy())
        if err:
            mine[0] = 1
        outs = [torch.empty_like(mine) for _ in range(self.m.world)]
        try:
            work = dist.all_gather(outs, mine, group=self.m.ctl, async_op=True)
        except Exception as e:  # noqa: BLE001
            raise _RankLost(str(e)) from e
        return _Agree(rno, list(items), err, info, works, outs, work, nck)

    def _finish_agree(self, ag: "_Agree") -> None:
        try:
            ag.work.wait()
        except Exception as e:  # noqa: BLE001 - a dead or stuck peer
            raise _RankLost(str(e)) from e
        me = self.m.rank
        meta = []
        for r, x in enumerate(ag.items):
            st = int(ag.outs[r][0])
            if x is None:
                meta.append((None, "", b""))
            elif st != 0:
                meta.append((x, ag.err if r == me and ag.err else
                             f"rank {self.m.granks[r]}: fetch failed (round {ag.rno})", b""))
            else:
                meta.append((x, "", ag.outs[r][1:1 + ag.nck[r]].numpy().tobytes()))
        fatal, _, recv = self._apply_meta(meta, ag.info)
        if self.unagreed:
            self.unagreed.pop(0)  # rounds are agreed in order
        if fatal:
            self._settle_received()
            raise SwarmPullError("; ".join(sorted(set(fatal))))
        if recv:
            ev = self._hash_received(recv, ag.works)
            if ev is not None:
                self.pending_events.append((ev, recv))
        elif not self.cuda:
            for w in ag.works:
                w.wait()

    # -- main loop ----------------------------------------------------------------------------
    def run(self):
        self.round_no = 0
        self.pending_events: list = []   # (event, items) of received rounds not yet known to be hashed
        self.unagreed: list = []
        for f in self.fetchers:  # (the tables are zeroed before any fetch pipeline writes them)
            f.order_after(getattr(self, "tables_ready", None))
        streamed = self.streamed
        while True:
            try:
                if streamed:
                    streamed = False
                    self._rounds_streamed()
                    if any(self.queue):
                        # reassigned ranges follow on the synchronous loop: their exchanges must land
                        # after the streamed ones that wrote the same regions (with a failed owner's
                        # bytes) on other streams
                        self._settle_received()
                        if self.cuda:
                            torch.cuda.synchronize(self.device)
                self._rounds()
                self._settle_received()
                return
            except _RankLost as e:
                self._recover(str(e))

    def _settle_received(self):
        for ev, items in self.pending_events:
            if ev is not None:
                _idle_wait(ev)
            self.have.update(items)
        self.pending_events = []

    def _fetch_one(self, fetcher, it, round_no: int):
        """Fetch item `it` (term ranges) into the arena: (error text, chunk sizes, source counters)."""
        P = self.plan
        if it is None:
            return "", b"", {}
        if it in self.have:  # a re-send after recovery: the bytes are here
            return "", self.item_lens[it], {}
        try:
            if (self.m.me, round_no) in self.fault["fail"]:
                raise RuntimeError(f"injected fetch failure (round {round_no})")
            a, b = self.items[it]
            res = fetcher.fetch(P.jobs(a, b, self.arena.data_ptr()), self.hashes, self.sizes)
            lens = b"".join(r["chunk_lens"] for r in res)
            info = {k: sum(r[k] for r in res) for k in ("fetched", "from_peer", "from_cdn", "from_cache")}
            return "", lens, info
        except Exception as e:  # noqa: BLE001 - reported through the all-gather
            return f"rank {self.m.me}: {type(e).__name__}: {e}", b"", {}

    def _pop_round(self) -> list:
        """Next round's item per rank: every rank pops the same queues at the same point."""
        return [q.pop(0) if q else None for q in self.queue]

    def _submit(self, nxt: list, round_no: int):
        from concurrent.futures import ThreadPoolExecutor
        if not hasattr(self, "_pool"):
            # HIP's current device is per thread: the pool's threads start on this rank's GPU
            init = (lambda: torch.cuda.set_device(self.device)) if self.cuda else None
            self._pool = ThreadPoolExecutor(max_workers=2, thread_name_prefix="zest-swarm-fetch", initializer=init)
        f = self.fetchers[round_no % len(self.fetchers)]
        return self._pool.submit(self._fetch_one, f, nxt[self.m.rank], round_no)

    def _join_fetch(self):
        """Wait for a fetch still in flight (its result is dropped: its item is re-queued), and cancel
        and drain the streamed items not yet collected."""
        if self._fut is not None:
            try:
                self._fut.result()
            except Exception:  # noqa: BLE001
                pass
            self._fut = None
        if getattr(self, "_tickets", None):
            self._tickets = []
            for f in self.fetchers:
                f.drain(cancel=True)

    def _rounds(self):
        P = self.plan
        me = self.m.rank
        nxt = self._pop_round()
        self.inflight_next = []
        if self.pipelined:
            self._fut = self._submit(nxt, self.round_no)
        while any(x is not None for x in nxt) or any(self.queue):
            this = nxt
            self.inflight = list(this)   # popped but not yet agreed (re-queued by _recover)
            it = this[me]
            if (self.m.me, self.round_no) in self.fault["exit"]:
                os._exit(1)  # fault injection: this rank dies mid-pull (tests)
            t = time.perf_counter()
            if self.pipelined:
                # the next round's items are assigned now, before this round is agreed (a range
                # re-queued by this round's failures is taken up one round later), and fetched on the
                # other pipeline while this round's fetch finishes
                nxt = self._pop_round()
                self.inflight_next = list(nxt)
                fut, self._fut = self._fut, None
                if any(x is not None for x in nxt):  # submitted BEFORE waiting: the two overlap
                    self._fut = self._submit(nxt, self.round_no + 1)
                # (nothing is in flight only when the previous pop found every queue empty, i.e.
                # `it` is None; a synchronous fetch covers anything else)
                err, lens, info = fut.result() if fut is not None else \
                    self._fetch_one(self.fetchers[self.round_no % len(self.fetchers)], it, self.round_no)
            else:
                err, lens, info = self._fetch_one(self.fetcher, it, self.round_no)
            self._mark("fetch_s", t)
            t = time.perf_counter()
            # (a group of one agrees with itself: no pickled round trip of every chunk size)
            meta = self._gather((it, err, lens)) if self.m.world > 1 else [(it, err, lens)]
            self._mark("agree_s", t)
            fatal, regions, recv = self._apply_meta(meta, info)
            self.inflight = []
            if fatal:
                self._join_fetch()
                self._settle_received()
                raise SwarmPullError("; ".join(sorted(set(fatal))))
            if self.m.world > 1 and any(hi > lo for lo, hi in regions):
                t = time.perf_counter()
                try:
                    works = self.xchg.exchange(regions, synced=True)
                    ev = self._hash_received(recv, works)
                except Exception as e:  # noqa: BLE001
                    raise _RankLost(str(e)) from e
                if ev is not None:
                    self.pending_events.append((ev, recv))
                self._mark("exchange_issue_s", t)
            self.round_no += 1
            if not self.pipelined:
                nxt = self._pop_round()
        self.inflight_next = []

    def _recover(self, why: str):
        """A rank was lost: rebuild the groups over the survivors and re-shard (see _Membership).
        Bounded: the whole recovery -- the membership vote, the RCCL abort, the device synchronize and
        the new groups -- runs under a deadline (ZEST_SWARM_RECOVER_TIMEOUT, default ctl timeout +
        60 s); a survivor that exceeds it exits with status 3 instead of hanging."""
        bound = float(os.environ.get("ZEST_SWARM_RECOVER_TIMEOUT", str(self.m.timeout_s + 60)))
        with _Deadline(bound, f"recovery from a lost rank ({why[:120]})"):
            self._recover_bounded(why)

    def _recover_bounded(self, why: str):
        t = time.perf_counter()
        old_world, old_granks = self.m.world, list(self.m.granks)
        # whatever the dead peer's exchanges left in flight is abandoned; only finished hashing counts
        done = []
        for ev, items in self.pending_events:
            if ev is None or ev.query():
                done += items
        self.have.update(done)
        self.pending_events = []
        self._join_fetch()  # (its range is re-queued below with the other unagreed ones)
        if self.cuda and getattr(self, "xchg", None) is not None:
            # exchange streams still waiting (on the GPU) for a dead owner's ready counter would never
            # finish: open every counter, abandoning those copies, before anything synchronizes
            self.xchg.release_signals()
        lost = self.m.rebuild()
        if not lost:
            raise SwarmPullError(f"collective failed but every rank is alive: {why}")
        self.stats["recovered_ranks"] += len(lost)
        if os.environ.get("ZEST_SWARM_FAULT_RECOVER") == "hang":  # fault injection (tests): a stuck abort/sync
            time.sleep(1e9)
        if self.cuda:
            torch.cuda.synchronize(self.device)
        # queues of the survivors, in their new order; everything of the lost ranks is re-planned
        keep = {g: self.queue[old_granks.index(g)] for g in self.m.granks}
        orphan = [x for i in lost for x in self.queue[i]]
        # ranges popped but never agreed (the failed round's, and the next round's already handed to
        # the other pipeline; the streamed phase's pending rounds): back to their owner, in order, or
        # orphaned
        for popped in list(reversed(getattr(self, "unagreed", []))) + [getattr(self, "inflight_next", []),
                                                                      getattr(self, "inflight", [])]:
            for i, x in enumerate(popped):
                if x is not None and x not in self.owner_of:
                    if old_granks[i] in keep:
                        if x not in keep[old_granks[i]]:
                            keep[old_granks[i]].insert(0, x)
                    else:
                        orphan.append(x)
        self.inflight = []
        self.inflight_next = []
        self.unagreed = []
        self.queue = [keep[g] for g in self.m.granks]
        # which items does every survivor hold?  (fetched ones, and received ones already hashed)
        fetched = sorted(self.owner_of)
        holds = self._gather(sorted(i for i in fetched if i in self.have))
        holders = {i: [r for r, h in enumerate(holds) if i in set(h)] for i in fetched}
        resend, refetch = [], list(orphan)
        for i in fetched:
            hs = holders[i]
            if len(hs) == self.m.world:
                continue
            if hs:
                resend.append((i, hs[0]))
            else:
                refetch.append(i)
                self.owner_of.pop(i, None)
        for i, r in resend:
            self.queue[r].insert(0, i)   # the holder sends it first (no fetch: its bytes are there)
        P = self.plan
        for i in sorted(set(refetch)):
            load = [sum(int(P.t_ulen[self.items[x][0]:self.items[x][1]].sum()) for x in q) for q in self.queue]
            q = min(range(self.m.world), key=lambda q: (load[q], q))
            self.queue[q].append(i)
        self.xchg = RoundExchange(self.arena, self.m.rank, self.m.world, self.m.data,
                                  "bcast" if self.m.world > 1 else "none")
        self._mark("recover_s", t)
        if self.m.rank == 0:
            print(f"[zest swarm] lost rank(s) {[old_granks[i] for i in lost]} of {old_world}: continuing on "
                  f"{self.m.world}; {len(resend)} range(s) re-sent, {len(set(refetch))} refetched", flush=True)

    # -- verification, repair, settle ---------------------------------------------------------
    def verify_files(self) -> list[int]:
        """Merkle file hashes on this rank; returns the indices of files failing on ANY rank."""
        P = self.plan
        nf = len(self.xet_files)
        if nf == 0:
            return []
        t = time.perf_counter()
        for it, ls in self.item_lens.items():
            a, _ = self.items[it]
            c0 = int(P.t_c0[a])
            arr = np.frombuffer(ls, dtype=np.uint32)
            self.lens[c0:c0 + len(arr)] = arr
        bad_local = np.zeros(nf, dtype=np.int32)
        if self.verify:
            empty = _core.xet_hex(_core.file_hash([]))
            idx = [i for i in range(nf) if P.file_t1[i] > P.file_t0[i]]
            for i in range(nf):
                if i not in idx and self.xet_files[i]["xet_hash"] != empty:
                    bad_local[i] = 1
            jobs = [(int(P.t_c0[P.file_t0[i]]), int(P.t_nck[P.file_t0[i]:P.file_t1[i]].sum())) for i in idx]
            sizes = torch.from_numpy(self.lens.astype(np.int64))
            sizes = sizes.to(self.device) if self.cuda else sizes
            if self.cuda:
                # (the received chunks' hashes first, waited for with sleeps: the Merkle copy below
                # would otherwise poll a core for the hashing backlog)
                done = torch.cuda.Event()
                done.record(self.verify_stream)
                _idle_wait(done)
                torch.cuda.current_stream(self.device).wait_stream(self.verify_stream)
            roots = ops.merkle_roots(self.hashes, sizes, jobs, file_hash=True).cpu().numpy()
            for j, i in enumerate(idx):
                if _core.xet_hex(roots[j].tobytes()) != self.xet_files[i]["xet_hash"]:
                    bad_local[i] = 1
        flags = torch.from_numpy(bad_local)
        try:
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=self.m.ctl)
        except Exception as e:  # noqa: BLE001
            raise _RankLost(str(e)) from e
        self._mark("verify_s", t)
        return [i for i in range(nf) if flags[i]]

    def repair(self, bad: list[int]) -> None:
        """Owners refetch the failed files' terms from the CDN; the ranges are re-sent to every rank
        over a plain RCCL broadcast (a broken peer mapping cannot corrupt them twice)."""
        t = time.perf_counter()
        P = self.plan
        badset = set(bad)
        for i in bad:
            for f in self.fetchers:
                f.settle(self.xet_files[i]["xet_hash"], False)
        # split each fetched item into its pieces inside bad files; the item's owner refetches them
        pieces = []   # (owner rank, a, b)
        for it, g in sorted(self.owner_of.items()):
            a, b = self.items[it]
            t_ = a
            while t_ < b:
                f = int(P.t_file[t_])
                e = min(b, int(P.file_t1[f]))
                if f in badset:
                    pieces.append((self.m.granks.index(g) if g in self.m.granks else 0, t_, e))
                t_ = e
        self.xchg.mode = "bcast" if self.m.world > 1 else self.xchg.mode
        per_rank = [[(a, b) for r, a, b in pieces if r == q] for q in range(self.m.world)]
        for k in range(max((len(p) for p in per_rank), default=0)):
            mine = per_rank[self.m.rank][k] if k < len(per_rank[self.m.rank]) else None
            err = ""
            if mine is not None:
                try:
                    self.fetcher.fetch(P.jobs(mine[0], mine[1], self.arena.data_ptr()), self.hashes, self.sizes,
                                       repair=True)
                except Exception as e:  # noqa: BLE001
                    err = f"rank {self.m.me}: {type(e).__name__}: {e}"
            errs = self._gather(err)
            if any(errs):
                raise zdev.VerifyError("repair fetch failed: " + "; ".join(e for e in errs if e))
            if self.m.world > 1:
                regions = [P.region(*per_rank[q][k]) if k < len(per_rank[q]) else (0, 0) for q in range(self.m.world)]
                works = self.xchg.exchange(regions)
                self.stats["resent_bytes"] += sum(hi - lo for q, (lo, hi) in enumerate(regions) if q != self.m.rank)
                recv = []
                for q in range(self.m.world):
                    if q != self.m.rank and k < len(per_rank[q]):
                        self.items.append(per_rank[q][k])
                        idx = len(self.items) - 1
                        a, b = per_rank[q][k]
                        self.item_lens[idx] = self._lens_of(a, b)
                        recv.append(idx)
                ev = self._hash_received(recv, works)
                if ev is not None:
                    ev.synchronize()
        self.stats["repaired_files"] += len(bad)
        self._mark("repair_s", t)

    def _lens_of(self, a: int, b: int) -> bytes:
        P = self.plan
        c0, c1 = int(P.t_c0[a]), int(P.t_c0[b - 1] + P.t_nck[b - 1])
        return self.lens[c0:c1].tobytes()

    def settle(self, ok_files: set[int]):
        mine = set()
        for it, g in self.owner_of.items():
            if g == self.m.me:
                mine.update(self.plan.files_of(*self.items[it]))
        for i in mine:
            for f in self.fetchers:
                f.settle(self.xet_files[i]["xet_hash"], i in ok_files)

    def plain(self) -> list[torch.Tensor]:
        """Non-Xet safetensors: rank 0 pulls them through the host path; broadcast to the others."""
        files = self.plain_files
        if not files:
            return []
        bufs = [ops.padded_empty(f["size"], self.device)[: f["size"]] if self.cuda
                else torch.empty(f["size"], dtype=torch.uint8) for f in files]
        err = ""
        if self.m.rank == 0:
            try:
                r = _core.pull(self.repo, self.revision, *self.fetcher.args[3:8], [f["path"] for f in files], True, 0,
                               self.repo_type)
                if r["failed_files"]:
                    raise SwarmPullError(f"host pull failed for {r['failed_files']} file(s)")
                for f, b in zip(files, bufs):
                    b.copy_(zdev.load_file(os.path.join(r["snapshot_dir"], f["path"]), self.device).view(torch.uint8))
                self.fetched_bytes += sum(f["size"] for f in files)
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
        err = self._bcast_from0(err)
        if err:
            raise SwarmPullError(f"non-Xet safetensors: {err}")
        for b in bufs:
            if b.numel() and self.m.world > 1:
                dist.broadcast(b, src=self.m.granks[0], group=self.m.data)
        return bufs

    def tensors(self, plain_bufs) -> dict[str, torch.Tensor]:
        out: dict[str, torch.Tensor] = {}
        views = [(f, self.arena[o:o + f["size"]]) for f, o in zip(self.xet_files, self.plan.file_off)]
        views += list(zip(self.plain_files, plain_bufs))
        views = [(f, buf) for f, buf in views if f["size"] >= 8]
        if not views:
            return out
        # every file's header length, then every header, in one device -> host copy each (two copies
        # per file cost a synchronizing round trip each: up to 60 ms per pull on a shared GPU)
        lens = torch.cat([buf[:8] for _, buf in views]).cpu().numpy().view("<u8")
        hlens = [min(int(h), int(f["size"]) - 8) for (f, _), h in zip(views, lens)]
        heads = torch.cat([buf[8:8 + h] for (_, buf), h in zip(views, hlens)]).cpu().numpy().tobytes()
        pos = 0
        for (f, buf), hlen in zip(views, hlens):
            head = int(hlen).to_bytes(8, "little") + heads[pos:pos + hlen]
            pos += hlen
            start, meta_ = zdev.parse_safetensors_header(head)
            for k, v in zdev.tensor_views(buf, start, meta_).items():
                if k in out:
                    raise ValueError(f"duplicate tensor {k} in {f['path']}")
                out[k] = v
        return out


# Per device: (pinned int64 offsets, pinned int32 sizes, device int64 offsets, device int32 sizes)
# with one slot per chunk of a pull (grown to the largest pull so far), for the received chunks'
# hash tables (_Swarm._hash_received).  A pull writes each chunk's slot once; the next pull reuses
# them only after its predecessor's verify waited for every hash.
_LAYOUT: dict = {}


def _layout_bufs(device, n: int):
    key = device.index
    b = _LAYOUT.get(key)
    if b is None or b[0].numel() < n:
        cap = max(int(n), 1 << 16)
        b = (torch.empty(cap, dtype=torch.int64).pin_memory(), torch.empty(cap, dtype=torch.int32).pin_memory(),
             torch.empty(cap, dtype=torch.int64, device=device), torch.empty(cap, dtype=torch.int32, device=device))
        _LAYOUT[key] = b
    return b


def _idle_wait(ev) -> None:
    """Wait for a torch.cuda.Event with short sleeps: Event.synchronize() polls a core for as long
    as the GPU takes (the one-GPU rehearsals share 16 CPUs between all ranks)."""
    d = 5e-6
    while not ev.query():
        time.sleep(d)
        d = min(d * 2, 1e-4)


def _merged_stats(parts: list) -> dict:
    """The pipelines' stats dicts summed (numbers) / first seen (other values)."""
    out: dict = {}
    for d in parts:
        for k, v in d.items():
            if isinstance(v, (int, float)) and not isinstance(v, bool) and isinstance(out.get(k, 0), (int, float)):
                out[k] = out.get(k, 0) + v
            else:
                out.setdefault(k, v)
    return out


# Pipelines kept by pulls made with reuse_pipeline=True, keyed by everything that shaped them: the
# next pull of the same repository in this process starts with its staging pinned and its Xet
# session up (the bench times repeated pulls; a long-lived loader pulling several revisions too).
_PIPELINES: dict = {}


# Arenas kept between pulls (reuse_arena): (arena, peer mappings or None, storage references when
# kept), keyed by device, world size, member ranks and whether the arena is peer-mapped.
_ARENAS: dict = {}


def _storage_refs(t: torch.Tensor) -> int:
    """References to t's storage (tensors viewing it, view bases, and the probe's own storage
    object)."""
    return int(torch._C._storage_Use_Count(t.untyped_storage()._cdata))


def _arena_in_use(entry) -> bool:
    """Whether any tensor besides the kept arena still views its storage (a caller's tensor of an
    earlier pull): more references than when the arena was kept."""
    return _storage_refs(entry[0]) > entry[2]


def adopt_arena(arena: torch.Tensor, mapped=None, group=None) -> None:
    """Seed the reuse_arena cache with an arena the caller already holds: the next reuse_arena=True
    pull over `group` of at most its size lands in it instead of allocating.  bench.py hands its
    engine's arena to the public-path row: freeing 141 GB and allocating it again costs the driver's
    reclaim -- and the engine's arena is peer-imported, and an imported VMM allocation is not returned
    before the importing process exits (profiles/r6/vmm_release_r6h_r6i/).  (`mapped`: unused; the
    public path exchanges through its own windows.)"""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    granks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(world))
    dev = arena.device.index if arena.device.type == "cuda" else -1
    _ARENAS[(dev, world, granks)] = (arena, None, _storage_refs(arena))


# Memberships kept by reuse_pipeline pulls (control / data groups, heartbeat), keyed by the group's
# ranks, backend and device.
_MEMBERS: dict = {}


def release_pipelines() -> None:
    """Drop the pipelines kept by reuse_pipeline=True pulls (their pinned staging is freed) and the
    arenas kept by reuse_arena=True pulls."""
    _PIPELINES.clear()
    for m in _MEMBERS.values():
        m.close()
    _MEMBERS.clear()
    _ARENAS.clear()


def _stats_delta(now: dict, base: dict) -> dict:
    """Counters of `now` minus `base` (numbers; nested dicts recursively; other values as in now)."""
    out = {}
    for k, v in now.items():
        b = base.get(k)
        if isinstance(v, dict):
            out[k] = _stats_delta(v, b if isinstance(b, dict) else {})
        elif isinstance(v, (int, float)) and not isinstance(v, bool) and isinstance(b, (int, float)):
            out[k] = v - b
        else:
            out[k] = v
    if "p2p_ratio" in out:
        tot = sum(out.get(k, 0) for k in ("bytes_from_cache", "bytes_from_peer", "bytes_from_cdn"))
        out["p2p_ratio"] = round(out.get("bytes_from_peer", 0) / tot, 4) if tot else 0.0
    return out


def _parallel_map(fn, items, threads: int):
    if not items:
        return []
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(threads, len(items))) as ex:
        return list(ex.map(fn, items))


def swarm_pull(repo: str, revision: str = "main", group=None, device=None, *, p2p: bool = True, peers=None,
               tracker=None, dht: bool = True, dht_bootstrap=None, repo_type: str = "model",
               verify_received: bool = True, staging_bytes: int = 1 << 30, threads: int = 16,
               round_bytes: int | None = None, exchange: str = "auto",
               stats: dict | None = None, reuse_pipeline: bool | None = None,
               possession: bool | None = None, reuse_arena: bool | None = None,
               files_out: dict | None = None) -> dict[str, torch.Tensor]:
    """Collective over `group`: returns {tensor_name: tensor} on this rank's device, every rank the
    full set (views into one arena per rank).  `exchange`: "auto" (measured at setup, cached per
    process) or one of p2p / bcast / allgather / ipc / xgmi.  `round_bytes` (default
    ZEST_SWARM_ROUND_MB, 1024 MiB): per-rank bytes per pipeline round.  `stats`, if given, is filled
    with this rank's numbers: bytes fetched / received, the exchange mode and its autotune times,
    per-phase seconds (with cross-round pipelining, `fetch_s` is the time spent waiting for a round's
    fetch to finish, not the fetches' own duration), re-shards and recovered ranks.

    `possession` (default ZEST_SWARM_POSSESSION, on): before sharding, every rank reports which terms
    its xorb cache already covers and holders own those terms (assign_owners) -- a rank with the
    whole model cached is the node's seeder.  `reuse_pipeline` (default ZEST_SWARM_REUSE, off): keep
    the fetch pipelines (pinned staging, Xet session) for the next pull of the same repository in
    this process; release_pipelines() frees them.  `reuse_arena`: True -- the pull lands in the
    arena kept from this process's previous pull over the same group (large enough) instead of a
    fresh one, overwriting that pull's tensors (bench.py's repeated pulls; kept until the next pull
    or release_pipelines()); None / False (default) -- a fresh arena, an ordinary device allocation
    that is freed once the caller drops the returned tensors.  At N > 1 the peer-mapped exchanges
    read the owners' exchange windows (fixed buffers of ZEST_SWARM_WINDOW_SLOTS x
    ZEST_SWARM_WINDOW_MB per rank, mapped into the group once per process), never a peer's arena:
    a released VMM import is not returned by the HIP runtime until the importing process exits
    (profiles/r6/vmm_release_r6h_r6i/).  `files_out`, if given, receives {path: uint8 tensor} --
    every pulled safetensors file's verified bytes (views of the arena), e.g. for writing a
    snapshot."""
    if reuse_pipeline is None:
        reuse_pipeline = os.environ.get("ZEST_SWARM_REUSE", "0") == "1"
    if os.environ.get("ZEST_SWARM_STAGING_MB"):  # per-slot staging of the fetch pipelines (A/B knob)
        staging_bytes = int(os.environ["ZEST_SWARM_STAGING_MB"]) << 20
    if possession is None:
        possession = os.environ.get("ZEST_SWARM_POSSESSION", "1") != "0"
    if round_bytes is None:
        round_bytes = int(os.environ.get("ZEST_SWARM_ROUND_MB", "1024")) << 20
    if exchange not in ("auto",) + EXCHANGE_MODES:
        raise ValueError(f"exchange={exchange!r}")
    sw = _Swarm(repo, revision, group, device, p2p=p2p, peers=peers, tracker=tracker, dht=dht,
                dht_bootstrap=dht_bootstrap, repo_type=repo_type, verify_received=verify_received,
                staging_bytes=staging_bytes, threads=threads, round_bytes=round_bytes, exchange=exchange,
                reuse=reuse_pipeline, possession=possession)
    sw.reuse_arena = reuse_arena
    sw._mark("init_s", sw.t0)
    ok = False
    try:
        while True:
            try:
                sw.listing_and_plan()
                sw.gather_possession()
                break
            except _RankLost as e:
                sw.m.rebuild()
                del e
        sw.allocate()
        t_s = time.perf_counter()
        sw.shard()
        sw._mark("shard_s", t_s)
        t_s = time.perf_counter()
        sw.setup_exchange()
        sw._mark("setup_exchange_s", t_s)
        t_pull = time.perf_counter()
        sw.t_pull = t_pull
        sw.run()
        for f in sw.fetchers:
            f.drain()  # (streamed items: every one was waited for; their events go, the timeline is made)
        if sw.cuda:
            torch.cuda.synchronize(sw.device)
        sw._mark("pull_s", t_pull)
        round_mode = sw.xchg.mode
        bad = sw.verify_files()
        sw.stats["first_verify_bad_files"] = len(bad)
        for _ in range(2):
            if not bad:
                break
            sw.repair(bad)
            bad = sw.verify_files()
        nf = len(sw.xet_files)
        t_t = time.perf_counter()
        sw.settle(set(range(nf)) - set(bad))
        if bad:
            raise zdev.VerifyError(f"rank {sw.m.me}: files failed their Xet hash after repair: "
                                   f"{[sw.xet_files[i]['path'] for i in bad]}")
        plain = sw.plain()
        out = sw.tensors(plain)
        if files_out is not None:
            for f, o in zip(sw.xet_files, sw.plan.file_off):
                files_out[f["path"]] = sw.arena[o:o + f["size"]]
            for f, b in zip(sw.plain_files, plain):
                files_out[f["path"]] = b
        if sw.cuda:
            torch.cuda.synchronize(sw.device)
        sw._mark("tensors_s", t_t)
        if stats is not None:
            total = sum(f["size"] for f in sw.xet_files) + sum(f["size"] for f in sw.plain_files)
            wall = time.perf_counter() - sw.t0
            stats.update(
                files=len(sw.xet_files) + len(sw.plain_files), fetched_bytes=sw.fetched_bytes,
                received_bytes=total - sw.fetched_bytes, total_bytes=total,
                p2p_ratio=(total - sw.fetched_bytes) / total if total else 0.0,
                rounds=sw.round_no, planned_rounds=sw.n_rounds_planned, items=len(sw.items),
                round_bytes=getattr(sw, "round_bytes_used", sw.round_bytes),
                exchange=round_mode, repair_exchange=sw.xchg.mode if sw.stats["repaired_files"] else None,
                exchange_autotune_s={k: round(v, 4) for k, v in sw.xchg.times.items()},
                peer_mapped=sw.xchg.mapped, world=sw.m.world, seconds=round(wall, 4),
                GBps=round(total / wall / 1e9, 4) if wall > 0 else 0.0, phases=dict(sw.times),
                fetch_stats=_stats_delta(_merged_stats([f.stats() for f in sw.fetchers if f.parent is None]),
                                         sw.stats_base),
                pipelined=sw.pipelined, streamed=sw.streamed, item_ready_s=getattr(sw, "item_ready_s", []),
                held_bytes=sw.held_bytes[sw.m.rank], share_bytes=sw.share_bytes[sw.m.rank],
                possession=list(sw.held_bytes), reused_pipeline=sw.reused,
                cache_writer=sw.fetcher.cache_writer(), device_timeline=sw.fetcher.timeline(),
                alloc=getattr(sw, "alloc_info", {}), **sw.stats)
        ok = True
        return out
    finally:
        if not ok and sw.cuda and getattr(sw, "xchg", None) is not None:
            # a failed pull may leave exchange streams waiting for counters that will never move:
            # open them before anything below synchronizes (the page is not reused)
            sw.xchg.release_signals()
        if getattr(sw, "_recon_warm", None) is not None:
            sw._recon_warm.join()
        if getattr(sw, "_fut", None) is not None:
            try:
                sw._fut.result()
            except Exception:  # noqa: BLE001 - the pull already failed
                pass
        if getattr(sw, "_pool", None) is not None:
            sw._pool.shutdown(wait=True)
        for f in getattr(sw, "fetchers", [sw.fetcher]):
            try:
                f.drain(cancel=not ok)  # (streamed items: every one was waited for unless the pull failed)
            except Exception:  # noqa: BLE001 - the pull already failed
                if ok:
                    raise
            f.join()
        if ok and sw.reuse and sw.m.epoch == 0:
            _MEMBERS[sw.member_key] = sw.m
        else:
            sw.m.close()
        if ok and sw.reuse:
            _PIPELINES[sw.reuse_key] = sw.fetchers
