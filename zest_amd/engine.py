"""Device pull engine: fetched xorb runs -> HBM arena (decode + verify) -> intra-node swarm exchange.

One process per GPU.  Each rank owns a contiguous, byte-balanced share of the model's
reconstruction terms (SURVEY §2.E P1 "term-parallel fetch", sharded by owner rank) and streams it
in rounds through a pinned-host -> HBM staging ring:

    lane k % 2  : hipMemcpyAsync(origin span k -> staging[k % 4])            (CDN/PCIe ingest)
                  -> index_terms -> place (copy | LZ4/BG4 decode) -> chunk hashes  (zest_amd.ops)
    RCCL        : round-k regions replicated over xGMI (batched p2p, coalesced broadcasts or slab
                  all-gather, whichever autotune_exchange measured fastest), overlapped with round
                  k+1 ingest (every GPU acts as a BitTorrent peer)
    verify      : chunks received from peers are BLAKE3-hashed on a side stream as each round lands,
                  so every rank hashes its whole replica itself (no peer's hashes are trusted)
    end         : Merkle file hashes on every rank (K2) -> compare with the repository's published
                  file hashes -> error all-reduce (C3)

The reference's equivalent is parallel_download.zig:91-204 (16 concurrent term fetches, batch
barrier, ordered writes) plus swarm.zig's peer fallback; here the "peers" of one node are GPUs and
the payload never bounces through the host after ingest.  The origin (what a CDN would have
returned for each term's url_range) lives in pinned host memory, so the measured pipeline is
everything zest does after bytes arrive from the network.
"""
from __future__ import annotations

import collections
import ctypes
import os
import time
from dataclasses import dataclass

import numpy as np
import torch

from . import _core, ops
from .synthetic import SyntheticWorld

from .parallel.exchange import (EXCHANGE_MODES, PEER_MAPPED_MODES, PeerArenas, RoundExchange,  # noqa: F401
                                _import_vmm_peers, _vmm_check, _vmm_mark, map_peer_arenas, role_stream)
from .parallel.exchange import StreamJoin as _StreamJoin  # noqa: F401


@dataclass
class RoundWork:
    term_a: int          # index range into world.terms (this rank's terms in this round)
    term_b: int
    c0: int              # first global chunk
    n_chunks: int
    span_off: int        # offset of the round's bytes in this rank's origin store
    span_len: int
    region: tuple        # arena [lo, hi) produced by this rank this round
    terms_dev: torch.Tensor | None = None  # TERM_DTYPE records (src relative to the staging slot)
    terms_host: np.ndarray | None = None   # the same records on the host (host header walk)
    table_off: int = 0                     # byte offset of the round's chunk records in a host table
    compressed: bool = True                # any chunk of the round stored LZ4/BG4 (decoder launch needed)


# Pinned allocations kept for reuse by the next OriginStore of this process (capacity, pointer).
# Pinning ~141 GB again after freeing it ran the following pull's H2D at 53.1 instead of 56.9 GB/s
# (bench.py, second data mode; profiles/bench70b_modes_r3.md), so a process that pulls several
# worlds pins once, sized by `reserve`.
_PINNED_POOL: list[tuple[int, int]] = []


# Device staging buffers of closed pullers, reused by the next one (same process, same device).
_STAGING_POOL: list[torch.Tensor] = []


def _staging_take(nbytes: int, device: torch.device) -> torch.Tensor:
    """A staging buffer of at least nbytes (rounded up to 64 MiB so worlds of nearly equal round
    sizes share the buffers)."""
    nbytes = -(-max(1, nbytes) // (64 << 20)) * (64 << 20)
    if device.type == "cuda":
        for i, t in enumerate(_STAGING_POOL):
            if t.device == device and t.numel() >= nbytes:
                return _STAGING_POOL.pop(i)
    return ops.padded_empty(nbytes, device)


_role_stream = role_stream

def release_pinned_pool() -> None:
    """Free the pinned buffers kept by closed OriginStores."""
    _STAGING_POOL.clear()
    H = ops.hip() if _PINNED_POOL else None
    while _PINNED_POOL:
        H.host_free(_PINNED_POOL.pop()[1])


def pinned_take(nbytes: int) -> tuple[int, int]:
    """(cap, ptr) of pinned host memory of at least nbytes: a pooled buffer, else a new one."""
    need = max(1, int(nbytes))
    hit = next((i for i, (cap, _) in enumerate(_PINNED_POOL) if cap >= need), None)
    if hit is not None:
        return _PINNED_POOL.pop(hit)
    release_pinned_pool()  # too small: give the pages back before pinning more
    return need, ops.hip().host_malloc(need)


def pinned_give(cap: int, ptr: int) -> None:
    """Return a pinned_take buffer to the pool (freed by release_pinned_pool)."""
    if ptr:
        _PINNED_POOL.append((int(cap), int(ptr)))


class OriginStore:
    """Pinned host memory holding the CDN response bytes for this rank's terms.  `reserve` (bytes)
    over-allocates so a later store of another world can reuse the same pinned pages.  `adopt` =
    (cap, ptr): take over a pinned buffer that already holds the bytes (a world build's
    serialized store) instead of allocating."""

    def __init__(self, nbytes: int, device: torch.device, reserve: int = 0, adopt=None):
        self.n = int(nbytes)
        self.device = device
        if device.type == "cuda":
            self._H = ops.hip()
            need = max(1, self.n)
            if adopt is not None:
                self.cap, self.ptr = int(adopt[0]), int(adopt[1])
                if self.cap < need:
                    raise ValueError("adopted origin buffer too small")
            else:
                self.cap, self.ptr = pinned_take(max(need, int(reserve)))
            self.array = np.ctypeslib.as_array((ctypes.c_uint8 * need).from_address(self.ptr))
        else:
            self._H = None
            self.array = np.empty(max(1, self.n), dtype=np.uint8)
            self.ptr = self.array.ctypes.data

    def close(self):
        if self._H is not None and self.ptr:
            torch.cuda.synchronize(self.device)  # no queued H2D copy still reads these pages
            if os.environ.get("ZEST_PIN_POOL", "1") != "0":
                _PINNED_POOL.append((self.cap, self.ptr))
            else:
                self._H.host_free(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plan_rank_terms(world: SyntheticWorld, n_ranks: int, seeders: int | None = None) -> list[tuple[int, int]]:
    """Contiguous, byte-balanced split of the term list among the first `seeders` ranks (default:
    all); the remaining ranks own nothing and receive the whole model from peers (leechers)."""
    T = world.terms
    k = n_ranks if seeders is None else max(1, min(seeders, n_ranks))
    if k < n_ranks:
        own = plan_rank_terms(world, k)
        return own + [(len(T), len(T))] * (n_ranks - k)
    from .parallel.split import even_bounds  # (the same cut as swarm_pull's owners)
    bounds = even_bounds(T["ulen"], n_ranks)
    return [(bounds[r], bounds[r + 1]) for r in range(n_ranks)]


HEAD_TAPER = (0.25, 0.5)        # first rounds, as fractions of a full round
TAIL_TAPER = (0.5, 0.25, 0.125)  # last rounds


def round_weights(share_bytes: int, round_bytes: int, taper: bool = True) -> list[float]:
    """Relative sizes of one rank's rounds.  Full rounds are at most `round_bytes`; with `taper`
    the first and last rounds shrink geometrically: nothing overlaps the first round's H2D and
    nothing overlaps the last round's exchange + verification, so those two rounds are the
    pipeline's head and tail (at 8 GPUs a 1 GiB tail is ~20 ms of xGMI traffic per ~0.35 s step,
    a 128 MiB one ~2.5 ms)."""
    n = max(1, -(-share_bytes // round_bytes))
    if not taper or n < 4:
        return [1.0] * n
    mid = max(1, -(-int(share_bytes - (sum(HEAD_TAPER) + sum(TAIL_TAPER)) * round_bytes) // round_bytes))
    return list(HEAD_TAPER) + [1.0] * mid + list(TAIL_TAPER)


def split_rounds(world: SyntheticWorld, a: int, b: int, weights) -> list[tuple[int, int]]:
    """Cut terms [a, b) into len(weights) rounds of (whole-term) byte sizes ~ proportional to
    `weights` (an int n means n equal rounds)."""
    T = world.terms
    if isinstance(weights, int):
        weights = [1.0] * weights
    n_rounds = len(weights)
    if b <= a:
        return [(a, a)] * n_rounds
    cu = np.cumsum(T["ulen"][a:b].astype(np.float64))
    total = cu[-1]
    frac = np.cumsum(np.asarray(weights, dtype=np.float64))
    frac /= frac[-1]
    cuts = [a]
    for k in range(1, n_rounds):
        cuts.append(a + int(np.searchsorted(cu, total * frac[k - 1], side="left")) + 1)
    cuts.append(b)
    cuts = np.maximum.accumulate(np.minimum(np.array(cuts), b))
    return [(int(cuts[k]), int(cuts[k + 1])) for k in range(n_rounds)]


class DevicePuller:
    def __init__(self, world: SyntheticWorld, arena: torch.Tensor, rank: int = 0, n_ranks: int = 1,
                 round_bytes: int = 1 << 30, slots: int = 3, group=None, exchange: str = "p2p",
                 seeders: int | None = None, origin_reserve: int = 0):
        self.world = world
        self.arena = arena
        self.device = arena.device
        self.rank, self.n_ranks = rank, n_ranks
        self.group = group
        self._exchange_mode0 = exchange
        self._ipc_done: dict = {}  # peer-mapped modes: round k's kernels done on this rank
        self._rx = _core.trace.roctx_enabled()  # ZEST_ROCTX=1: one roctx range per round (host-side issue)
        self.is_cuda = self.device.type == "cuda"
        T = world.terms
        self.rank_terms = plan_rank_terms(world, n_ranks, seeders)
        max_share = max((int(T["ulen"][a:b].sum()) for a, b in self.rank_terms), default=0)
        self.round_weights = round_weights(max_share, round_bytes, os.environ.get("ZEST_ROUND_TAPER", "1") != "0")
        self.n_rounds = len(self.round_weights)
        # rounds[k][r] = (a, b) term range for rank r in round k
        per_rank = [split_rounds(world, a, b, self.round_weights) for a, b in self.rank_terms]
        self.rounds_all = [[per_rank[r][k] for r in range(n_ranks)] for k in range(self.n_rounds)]
        # Pipeline shape (see the streams below): "copy" when any chunk is stored compressed.
        compressed = bool(world.chunk_clen is not None and np.any(world.chunk_clen < world.chunk_len))
        pipeline = os.environ.get("ZEST_PIPELINE", "copy" if compressed else "lanes")
        # The bf16 (copy) pipeline walks each round's chunk headers on the device (k_index_terms,
        # ~0.6 ms per 1 GiB round on its lane, under the round's ~18 ms H2D copy).  Round 4 tried a
        # host walk whose records rode the round's H2D copy: 58.4 vs 64.3 GB/s on the 70B bench
        # (profiles/r4/bench_ride_records_r4c.log), so it was removed.
        # this rank's origin layout: its terms' serialized bytes back to back, in order
        a_r, b_r = self.rank_terms[rank]
        ser_len = T["ser_len"][a_r:b_r].astype(np.int64)
        self.term_origin_off = np.concatenate([[0], np.cumsum(ser_len)]).astype(np.int64)  # relative to a_r
        # A one-rank origin is every chunk serialized in chunk order: exactly what a compressed world
        # build leaves in its pinned ser_store, so adopt those bytes instead of compressing again
        # (the second k_lz4_compress pass was ~40 s of the 70B bench's setup).
        ser = getattr(world, "serialized", None)
        adopt = None
        if (ser is not None and self.is_cuda and a_r == 0 and b_r == len(T)
                and int(ser[2]) == int(self.term_origin_off[-1])):
            adopt = (int(ser[1]), int(ser[0]))
            world.serialized = None
        self.origin = OriginStore(int(self.term_origin_off[-1]), self.device, origin_reserve, adopt=adopt)
        self.origin_prebuilt = adopt is not None
        self.rounds: list[RoundWork] = []
        max_span, max_terms, max_chunks = 0, 1, 1
        for k in range(self.n_rounds):
            a, b = self.rounds_all[k][rank]
            span_off = int(self.term_origin_off[a - a_r])
            span_len = int(self.term_origin_off[b - a_r] - self.term_origin_off[a - a_r])
            if b > a:
                c0 = int(T["c0"][a])
                nck = int(T["c1"][b - 1] - c0)
                rec = np.zeros(b - a, dtype=ops.TERM_DTYPE)
                rec["src"] = self.term_origin_off[a - a_r:b - a_r] - self.term_origin_off[a - a_r]
                rec["src_len"] = T["ser_len"][a:b]
                rec["dst"] = T["dst"][a:b]
                rec["chunk_base"] = T["c0"][a:b] - c0
                rec["n_chunks"] = T["c1"][a:b] - T["c0"][a:b]
                rec["ulen"] = T["ulen"][a:b]
                region = (int(T["dst"][a]), int(T["dst"][b - 1] + T["ulen"][b - 1]))
                terms_dev = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)
            else:
                c0, nck, rec, region, terms_dev = 0, 0, None, (0, 0), None
            comp = bool(world.chunk_scheme is not None and b > a and world.chunk_scheme[c0:c0 + nck].any())
            self.rounds.append(RoundWork(a, b, c0, nck, span_off, span_len, region, terms_dev, rec,
                                         sum(r.n_chunks for r in self.rounds) * ops.CHUNK_DTYPE.itemsize, comp))
            max_span = max(max_span, span_len)
            max_terms = max(max_terms, b - a)
            max_chunks = max(max_chunks, nck)
        self.regions = [[self._region(k, r) for r in range(n_ranks)] for k in range(self.n_rounds)]
        # intra-node replication of each round's regions (zest_amd.parallel.exchange)
        self.xchg = RoundExchange(arena, rank, n_ranks, group, self._exchange_mode0,
                                  gather_capacity=max((hi - lo for regs in self.regions for lo, hi in regs), default=0))
        # Two compute lanes take alternate rounds.  Round k runs entirely on lane k % 2: its H2D copy
        # into staging slot k % slots, then its kernels.  With an even slot count a slot is reused
        # only by the same lane, in stream order, so the pipeline needs no events, and there is
        # always a copy queued behind the other lane's kernels: the two lanes' copies keep PCIe busy
        # (56.9 GB/s vs 56.2 for one copy stream gated by slot-free events, 70B pull,
        # tools/step_times.py), while round k+1's kernels fill the CUs left idle in the tail of
        # round k's decode (a 1 GiB round is ~2 chunks per resident wave).
        self.slots = max(2, slots + (slots & 1))
        self.staging = [_staging_take(max_span, self.device) for _ in range(min(self.slots, self.n_rounds))]
        self.ws_lanes = [ops.IngestWorkspace(self.device, max_terms, max_chunks) for _ in range(2)]
        self.hashes = torch.zeros((world.n_chunks, 32), dtype=torch.uint8, device=self.device)
        self.sizes = torch.from_numpy(world.chunk_len.astype(np.int64)).to(self.device)
        self.expected = torch.from_numpy(world.file_hashes.copy()).to(self.device)
        self.err = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.jobs = world.merkle_jobs()
        if self.is_cuda:
            H = ops.hip()
            rec = np.zeros(len(self.jobs), dtype=ops.MERKLE_JOB_DTYPE)
            rec["leaf_base"] = [j[0] for j in self.jobs]
            rec["n_leaves"] = [j[1] for j in self.jobs]
            rec["want_file_hash"] = 1
            self.jobs_dev = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)
            self.merkle_sb = H.merkle_scratch_bytes(max(j[1] for j in self.jobs), len(self.jobs))
            self.merkle_scratch = torch.empty(self.merkle_sb, dtype=torch.uint8, device=self.device)
            self.roots = torch.empty((len(self.jobs), 32), dtype=torch.uint8, device=self.device)
            # Ingest (H2D copies, index/place/hash of this rank's rounds) is on the critical path:
            # its streams run at high priority; the receive-side verification (verify_stream) stays
            # at normal priority and fills whatever the ingest and the exchange leave idle.
            try:
                hi = int(torch.cuda.Stream.priority_range()[1])  # (least, greatest); lower = more urgent
            except Exception:
                hi = -1
            self.lane_stream = _role_stream(self.device, "lane", hi)
            self.side_stream = _role_stream(self.device, "side", hi)
            copy_stream = _role_stream(self.device, "copy", hi)  # created in a fixed order for every world
            # Pipeline shape.  "lanes": each round's H2D copy rides its compute lane (above; best when
            # the kernels are short next to the copy: raw chunks, 56.9 vs 56.2 GB/s).  "copy": one
            # copy stream issues every round's H2D back to back, gated only by slot-free events, so
            # PCIe never waits behind a lane's kernels -- needed when rounds decode LZ4/BG4 (a 1 GiB
            # bf16 round decodes in ~13 ms against ~16 ms of H2D; in "lanes" the two lanes drift
            # into copying together and decoding together, leaving PCIe idle: 54.3 vs 64.3 GB/s).
            # Default: "copy" when any chunk is stored compressed; ZEST_PIPELINE overrides.
            self.pipeline = pipeline
            if self.pipeline not in ("lanes", "copy"):
                raise ValueError(f"ZEST_PIPELINE={self.pipeline!r}: expected 'lanes' or 'copy'")
            if self.pipeline == "copy":
                self.copy_stream = copy_stream
                self.h2d_done = [torch.cuda.Event() for _ in self.staging]
                self.slot_free = [torch.cuda.Event() for _ in self.staging]
        # Host run-ahead bound: step() issues ~10 HIP commands per round (~1300 per 70B step) in ~10 ms
        # and returns, so a caller looping over step() without syncing queues thousands of commands
        # over many steps, and past ~10 steps queued the HIP runtime fed the device measurably slower
        # (bench.py 20 steps: 51-52.6 GB/s vs 56.2 with 10; tools/step_times.py).  step() therefore
        # waits until at most `steps_ahead` earlier steps are still in flight (0 = unbounded).
        self.steps_ahead = int(os.environ.get("ZEST_STEPS_AHEAD", "1"))
        # Peer-mapped exchanges: rounds queued past round k before the host waits for k to be readable
        # (ZEST_IPC_LAG, >= 1).  With both ranks on one GPU (the only multi-rank run a one-GPU box
        # allows) lag 1 and 2 measure the same, 279 / 294 ms per 8B bf16 step within that run's spread
        # (profiles/r5/rehearsal_n2_r5t/); 2 keeps a copy queued on a rank that owns its PCIe link.
        self.ipc_lag = max(1, int(os.environ.get("ZEST_IPC_LAG", "2")))
        self._inflight: collections.deque = collections.deque()
        # Header walk on the host (ZEST_HOST_INDEX, default on): the origin bytes are in host memory,
        # where the walk's pointer chase (chunk i+1's header position depends on chunk i's length)
        # runs at DRAM latency; each round's chunk records then reach the GPU with its copy, and the
        # lane runs only place + hash (the device walk, k_index_terms, was a serial 0.84 ms HBM
        # pointer chase per 1 GiB round and the largest kernel in the profile).  Pinned record
        # tables alternate by step parity, which is race-free while at most one earlier step is in
        # flight (steps_ahead == 1); otherwise, and inside a HIP graph, the device walk runs.
        # The copy pipeline keeps the device walk: a round's small record upload (host walk) would sit
        # on a lane or the copy stream between 1 GiB transfers, and the host blocked on it, leaving
        # one copy in flight at a time (BG4 bf16 70B: 53.5 / 59.2 GB/s with host records on the
        # copy stream / the lane, vs 64.3 with the device walk; profiles/pipeline_ab_r2.md).
        self.host_index = (self.is_cuda and self.steps_ahead == 1 and getattr(self, "pipeline", "lanes") == "lanes"
                           and os.environ.get("ZEST_HOST_INDEX", "1") != "0")
        if self.host_index:
            nbytes = max(1, sum(r.n_chunks for r in self.rounds) * ops.CHUNK_DTYPE.itemsize)
            self._tables = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self._step_no = 0
        self._graph = None        # one-GPU steps replayed from a HIP graph (capture_graph)
        self._capturing = False
        # Chunks this rank receives in each round, as contiguous index runs (one per sending peer):
        # every rank BLAKE3-hashes them as soon as they land, so each GPU verifies its whole replica
        # against the published Merkle file hashes without trusting any peer's hashes.
        self.recv_runs = [[] for _ in range(self.n_rounds)]
        for k in range(self.n_rounds):
            for p in range(n_ranks):
                a, b = self.rounds_all[k][p]
                if p != rank and b > a:
                    c0 = int(T["c0"][a])
                    self.recv_runs[k].append((c0, int(T["c1"][b - 1]) - c0))
        if self.is_cuda and n_ranks > 1:
            self.chunk_off_dev = torch.from_numpy(world.chunk_off.astype(np.int64)).to(self.device)
            self.chunk_len_dev = torch.from_numpy(world.chunk_len.astype(np.int32)).to(self.device)
            self.verify_stream = _role_stream(self.device, "verify")
            self._verify_scratch = ops.HashScratch(self.device)
            self._chunk_len_csum = np.concatenate([[0], np.cumsum(world.chunk_len, dtype=np.int64)])
        self.bytes_received = sum(hi - lo for k in range(self.n_rounds) for r, (lo, hi) in
                                  enumerate(self.regions[k]) if r != rank)
        self.bytes_ingested = int(self.term_origin_off[-1])

    def _region(self, k, r):
        a, b = self.rounds_all[k][r]
        T = self.world.terms
        if b <= a:
            return (0, 0)
        return (int(T["dst"][a]), int(T["dst"][b - 1] + T["ulen"][b - 1]))

    # ------------------------------------------------------------------------------------------
    def build_origin(self, pack_batch_bytes: int = 4 << 30) -> None:
        """Serialize this rank's terms ([header | payload]*) from the content in the arena into
        the pinned origin store (GPU pack kernel + D2H).  Untimed setup."""
        w = self.world
        T = w.terms
        a_r, b_r = self.rank_terms[self.rank]
        if b_r <= a_r or self.origin_prebuilt:
            return
        if not self.is_cuda:
            raise RuntimeError("CPU worlds build the origin from host contents (build_origin_host)")
        H = ops.hip()
        st = torch.cuda.current_stream(self.device).cuda_stream
        tmp = ops.padded_empty(min(pack_batch_bytes, self.origin.n) + (64 << 20), self.device)
        for rw in self.rounds:  # a round's span is contiguous in the origin
            t = rw.term_a
            while t < rw.term_b:
                base = int(self.term_origin_off[t - a_r])
                u = t
                while u < rw.term_b and self.term_origin_off[u + 1 - a_r] - base <= tmp.numel():
                    u += 1
                if u == t:
                    raise RuntimeError("term larger than pack batch")
                c0, c1 = int(T["c0"][t]), int(T["c1"][u - 1])
                ser = w.chunk_clen[c0:c1].astype(np.uint64) + np.uint64(8)
                out_off = (np.cumsum(ser) - ser).astype(np.uint64)
                w.pack_serialized(self.arena, c0, c1, tmp, out_off)
                n = int(self.term_origin_off[u - a_r] - base)
                at = rw.span_off + base - int(self.term_origin_off[rw.term_a - a_r])
                H.memcpy_async(self.origin.ptr + at, tmp.data_ptr(), n, st)
                torch.cuda.synchronize(self.device)
                t = u

    def build_origin_host(self, contents: dict[str, bytes]) -> None:
        w = self.world
        T = w.terms
        a_r, b_r = self.rank_terms[self.rank]
        start = {rw.term_a: rw.span_off for rw in self.rounds if rw.term_b > rw.term_a}
        pos = 0
        for t in range(a_r, b_r):
            pos = start.get(t, pos)  # each round's span starts at its own origin offset
            f = w.xet_files[int(T["file"][t])]
            data = contents[f.path]
            for c in range(int(T["c0"][t]), int(T["c1"][t])):
                rel = int(w.chunk_off[c]) - f.arena_off
                n = int(w.chunk_len[c])
                hdr = bytes([0, n & 255, (n >> 8) & 255, (n >> 16) & 255, 0, n & 255, (n >> 8) & 255, (n >> 16) & 255])
                self.origin.array[pos:pos + 8] = np.frombuffer(hdr, dtype=np.uint8)
                self.origin.array[pos + 8:pos + 8 + n] = np.frombuffer(data[rel:rel + n], dtype=np.uint8)
                pos += 8 + n

    # ------------------------------------------------------------------------------------------
    @property
    def exchange(self) -> str:
        """The intra-node exchange strategy (zest_amd.parallel.exchange); set, or picked by
        autotune_exchange."""
        return self.xchg.mode

    @exchange.setter
    def exchange(self, mode: str) -> None:
        self.xchg.mode = mode

    @property
    def exchange_times(self) -> dict:
        return self.xchg.times

    def _exchange(self, k: int, mode: str | None = None):
        """Replicate round k's regions to every rank.  Peer-mapped modes wait for
        this rank's round-k kernels (event recorded by step()), then a host barrier."""
        done = self._ipc_done.get(k)
        if isinstance(done, int):  # a ready-counter sequence number (signal_ready): GPU-side waits
            return self.xchg.exchange(self.regions[k], mode, seq=done)
        return self.xchg.exchange(self.regions[k], mode, ready=done)

    def enable_ipc(self, mapped: "PeerArenas | None" = None) -> bool:
        """Map every peer's arena into this process (HIP VMM / IPC) for the ``ipc`` / ``xgmi``
        exchanges.  Collective; True only if every rank mapped every peer.  Also shares the ranks'
        ready counters (RoundExchange.enable_signals), so a step's exchanges wait on the GPU for
        the owners' rounds instead of in a host event synchronize + barrier per round."""
        if not self.xchg.enable_ipc(mapped):
            return False
        self.xchg.enable_signals()
        return True

    def autotune_exchange(self, modes=EXCHANGE_MODES, max_rounds: int = 4) -> dict:
        """Time each exchange strategy over the first full-size rounds and keep the fastest (setup,
        untimed; RoundExchange.autotune)."""
        full = [k for k, w in enumerate(self.round_weights) if w == 1.0]  # time full-size rounds
        rounds = (full or list(range(self.n_rounds)))[:max_rounds]
        return self.xchg.autotune([self.regions[k] for k in rounds], modes)

    def _sync(self):
        if self.is_cuda:
            torch.cuda.synchronize(self.device)

    def _host_records(self, rw: RoundWork) -> int:
        """Host header walk of round rw's runs in the pinned origin into this step's pinned record
        table (error word set stream-ordered on the current stream); returns the records' address."""
        tab = self._tables[self._step_no & 1]
        rec_ptr = tab.data_ptr() + rw.table_off
        e = _core.index_runs(self.origin.ptr + rw.span_off, rw.span_len, rw.terms_host.ctypes.data,
                             rw.term_b - rw.term_a, rec_ptr, rw.n_chunks)
        if e:
            self.err.fill_(e)  # (stream-ordered, like the device walk's error word)
        return rec_ptr

    def _ingest_round(self, H, rw: RoundWork, src: torch.Tensor, ws, st: int) -> None:
        """Round rw on stream st: header walk (host or device), place/decode, BLAKE3 chunk hashes."""
        if rw.term_b <= rw.term_a:
            return
        nbytes = rw.n_chunks * ops.CHUNK_DTYPE.itemsize
        chunks = ws.chunks
        chunks_ptr = chunks.data_ptr()
        if self.host_index and not self._capturing:
            H.memcpy_async(chunks_ptr, self._host_records(rw), nbytes, st)
        else:
            chunks[:nbytes].zero_()
            ops.index_terms(H, src.data_ptr(), rw.span_len, rw.terms_dev.data_ptr(), rw.term_b - rw.term_a,
                            chunks_ptr, self.err.data_ptr(), st, None if self._capturing else ws)
        sp, sb = ws.hash_scratch.get(rw.n_chunks, rw.region[1] - rw.region[0])
        if ops.FUSED_INGEST:
            # decode (compressed rounds only) + ONE pass that places raw chunks and hashes every chunk
            H.ingest_chunks(src.data_ptr(), rw.span_len, self.arena.data_ptr(), self.arena.numel(), chunks_ptr,
                            rw.n_chunks, rw.compressed, self.err.data_ptr(), self.hashes.data_ptr() + 32 * rw.c0, 0, 0,
                            st, sp, sb)
            return
        H.place_chunks(src.data_ptr(), rw.span_len, self.arena.data_ptr(), self.arena.numel(), chunks_ptr,
                       rw.n_chunks, 0, self.arena.numel(), self.err.data_ptr(), st)
        H.hash_chunks(self.arena.data_ptr(), self.arena.numel(), chunks_ptr, rw.n_chunks,
                      self.hashes.data_ptr() + 32 * rw.c0, 0, 0, st, sp, sb)

    def capture_graph(self) -> bool:
        """One GPU: record a whole step (every round's H2D copy and index/place/hash kernels on the two
        compute lanes, the Merkle check) into one HIP graph, so a step is a single graph launch
        instead of ~1300 HIP calls from Python.  Collectives stay eager (N > 1 is not captured).
        Returns False, leaving eager steps, where capture is unavailable (ZEST_GRAPH=0, CPU, N > 1,
        or the runtime refuses).

        The step's stream shape captures as is: every round lives on one lane, so the graph has no
        cross-stream events (an earlier pipeline whose copy stream and lanes waited on each other
        crashed hipStreamEndCapture, ROCm 7: tools/experiments/graph_probe3.py X).  Host cost per step drops from
        ~1300 Python-issued HIP calls to one launch, but the graph's copy nodes ran slower (70B pull:
        51.2 GB/s, the same shape issued eagerly 56.9; profiles/hip_graph_r2.md), so bench.py uses it
        only with ZEST_GRAPH=1."""
        if not self.is_cuda or self.n_ranks > 1 or os.environ.get("ZEST_GRAPH", "1") == "0":
            return False
        self.step()  # eager pass: every buffer (hash scratch) exists before capture
        self._sync()
        g = torch.cuda.CUDAGraph()
        self._capturing = True
        try:
            with torch.cuda.graph(g):
                self.step()
        except Exception:  # noqa: BLE001 - fall back to eager steps
            self._capturing = False
            self._sync()
            return False
        self._capturing = False
        self._graph = g
        return True

    def step(self) -> dict:
        """One full pull of the model onto every rank.  Returns per-step stats."""
        import torch.distributed as dist
        dev = self.device
        if self.is_cuda and self.steps_ahead > 0 and not self._capturing:
            while len(self._inflight) > self.steps_ahead:
                self._inflight.popleft().synchronize()
        if self._graph is not None:
            self._graph.replay()
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(dev))
            self._inflight.append(done)
            return {"rounds": self.n_rounds, "graph": True}
        self.hashes.zero_()  # err is NOT reset: the first error of any step persists until check()
        self._step_no += 1
        works = []
        if self.is_cuda:
            H = ops.hip()
            main = torch.cuda.current_stream(dev)
            lanes = (self.lane_stream, self.side_stream)
            for ln in lanes:
                ln.wait_stream(main)  # hashes.zero_() above, and the caller's earlier work
            if self.n_ranks > 1 and self.xchg.signaled and self.exchange in PEER_MAPPED_MODES:
                # the peers' copies into this arena must land after the caller's own writes to it
                # (the warm-up poisons the arena on the main stream): r5v's first signaled
                # rehearsal lost that race in its second data mode (hash mismatch at index 0)
                self.xchg.order_after(main)
            for k, rw in enumerate(self.rounds):
                comp, ws = lanes[k % 2], self.ws_lanes[k % 2]
                src = self.staging[k % len(self.staging)]
                st = comp.cuda_stream
                if self._rx:
                    _core.trace.roctx_push(f"engine: round {k}")
                copy_mode = self.pipeline == "copy" and not self._capturing
                if copy_mode:
                    slot = k % len(self.staging)
                    with torch.cuda.stream(self.copy_stream):
                        self.copy_stream.wait_event(self.slot_free[slot])  # no-op before first use
                        if rw.span_len:
                            H.memcpy_async(src.data_ptr(), self.origin.ptr + rw.span_off, rw.span_len,
                                           self.copy_stream.cuda_stream)
                        self.h2d_done[slot].record(self.copy_stream)
                with torch.cuda.stream(comp):
                    if copy_mode:
                        comp.wait_event(self.h2d_done[slot])
                    elif rw.span_len:
                        H.memcpy_async(src.data_ptr(), self.origin.ptr + rw.span_off, rw.span_len, st)
                    self._ingest_round(H, rw, src, ws, st)
                    if copy_mode:
                        self.slot_free[slot].record(comp)
                    if self.n_ranks > 1:
                        if self.exchange in PEER_MAPPED_MODES:
                            # peers read round k once its kernels are done; wait for that only after
                            # rounds k+1 .. k+lag are queued, so the copy engine always has a round
                            # queued behind the one in flight while the host waits on the event and
                            # the host barrier (lag 1 left one copy queued: the barrier's wake-up
                            # skew became a PCIe gap every round)
                            if self.xchg.signaled:
                                self._ipc_done[k] = self.xchg.signal_ready(comp)
                            else:
                                self._ipc_done[k] = torch.cuda.Event()
                                self._ipc_done[k].record(comp)
                            if k >= self.ipc_lag:
                                j = k - self.ipc_lag
                                works += self._hash_received(j, self._exchange(j))
                        else:  # collectives wait for the issuing (this round's) stream
                            works += self._hash_received(k, self._exchange(k))
                if self._rx:
                    _core.trace.roctx_pop()
            main.wait_stream(self.lane_stream)
            main.wait_stream(self.side_stream)
            st = main.cuda_stream
            if self.n_ranks > 1 and self.exchange in PEER_MAPPED_MODES:
                for j in range(max(0, self.n_rounds - self.ipc_lag), self.n_rounds):
                    works += self._hash_received(j, self._exchange(j))
                self._ipc_done.clear()
            if self.n_ranks > 1:
                works.append(_StreamJoin(self.verify_stream))
        else:
            for k, rw in enumerate(self.rounds):
                if rw.term_b > rw.term_a:
                    span = torch.from_numpy(self.origin.array[rw.span_off:rw.span_off + rw.span_len])
                    rec = np.frombuffer(rw.terms_dev.numpy().tobytes(), dtype=ops.TERM_DTYPE)
                    ops.ingest_terms(span, self.arena, rec, self.hashes, hash_base=rw.c0)
                if self.n_ranks > 1:
                    works += self._hash_received(k, self._exchange(k))
        for w in works:
            w.wait()
        if self.is_cuda:
            H.merkle(self.hashes.data_ptr(), self.sizes.data_ptr(), self.jobs_dev.data_ptr(), len(self.jobs),
                     self.roots.data_ptr(), self.merkle_scratch.data_ptr(), self.merkle_sb, st)
            H.compare_hashes(self.roots.data_ptr(), self.expected.data_ptr(), len(self.jobs), self.err.data_ptr(), st)
            if self.steps_ahead > 0 and not self._capturing:
                done = torch.cuda.Event()
                done.record(main)
                self._inflight.append(done)
        else:
            roots = ops.merkle_roots(self.hashes, self.sizes, self.jobs)
            if not torch.equal(roots, self.expected):
                self.err.fill_((6 << 32) | int((roots != self.expected).any(1).nonzero()[0].item()))
        if self.n_ranks > 1:
            dist.all_reduce(self.err, op=dist.ReduceOp.MAX, group=self.group)
        return {"rounds": self.n_rounds}

    def check(self) -> None:
        ops.raise_on_error(self.err)

    def _hash_received(self, k: int, works: list) -> list:
        """Hash round k's chunks received from peers into this rank's own table as soon as the
        transfers land (side stream on the GPU, overlapped with later rounds).  Returns the works the
        caller still has to wait for: none once they were waited here (a gloo work must not be waited
        twice; on the GPU the caller's final join on the verify stream covers them)."""
        runs = self.recv_runs[k]
        if not runs:
            return works
        if not self.is_cuda:
            for w in works:
                w.wait()
            wd = self.world
            for c0, n in runs:
                self.hashes[c0:c0 + n] = ops.hash_ranges(self.arena, wd.chunk_off[c0:c0 + n], wd.chunk_len[c0:c0 + n])
            return []
        H = ops.hip()
        with torch.cuda.stream(self.verify_stream):
            for w in works:
                w.wait()  # the verify stream waits for round k's transfers
            for c0, n in runs:
                sp, sb = self._verify_scratch.get(n, self._run_bytes(c0, n))
                H.hash_ranges(self.arena.data_ptr(), self.chunk_off_dev.data_ptr() + 8 * c0,
                              self.chunk_len_dev.data_ptr() + 4 * c0, n, self.hashes.data_ptr() + 32 * c0,
                              ops.KEY_DATA, self.verify_stream.cuda_stream, sp, sb)
        return []

    def _run_bytes(self, c0: int, n: int) -> int:
        return int(self._chunk_len_csum[c0 + n] - self._chunk_len_csum[c0])

    def release_device(self) -> None:
        """Drop this puller's device buffers (arena view, staging, tables) but keep the pinned origin:
        bench.py's swarm row serves its CDN from the origin while swarm_pull allocates its own arena."""
        if self.is_cuda:
            torch.cuda.synchronize(self.device)
        self.arena = None
        self.staging = []
        self.hashes = self.sizes = self.expected = None
        self.ws_lanes = []
        self.xchg = None
        for k in ("merkle_scratch", "roots", "jobs_dev", "chunk_off_dev", "chunk_len_dev"):
            if hasattr(self, k):
                setattr(self, k, None)
        for rw in self.rounds:
            rw.terms_dev = None

    def close(self):
        if self.is_cuda:
            # queued H2D copies still read the pinned origin and kernels the staging buffers: the
            # next puller of this process reuses both, so nothing may be in flight when they go back
            torch.cuda.synchronize(self.device)
        self.origin.close()
        if self.is_cuda:
            _STAGING_POOL.extend(self.staging)  # the next puller of this process reuses them
            self.staging = []
