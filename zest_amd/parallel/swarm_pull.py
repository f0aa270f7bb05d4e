"""Intra-node swarm pull: every GPU of a node ends up with every tensor of a repository in its HBM,
while each Xet file crosses the network (peers / CDN / local xorb cache) exactly once.

    # one process per GPU (torchrun), backend "nccl" = RCCL over xGMI
    tensors = swarm_pull("meta-llama/Llama-3.1-70B")   # collective; every rank gets all tensors
    tensors = zest_amd.pull("meta-llama/Llama-3.1-70B", device="all")   # the same, public API

Each Xet-backed safetensors file has one owner rank (LPT split by size).  The pull runs in rounds
of one file per owner:

  fetch     the owner pulls its file device-direct (`_hip.DeviceXetPull`: compressed runs -> pinned
            staging -> GPU decode + BLAKE3 + Merkle check, with the native bridge's peer-quarantine /
            CDN-repair rules) -- or, on CPU process groups, through the host waterfall into memory
            (`_core.HostXetFetcher`); no snapshot is written either way
  agree     one small all_gather of (error, chunk sizes) per round: every rank learns which fetches
            worked and the chunk boundaries the owner parsed from the xorb headers
  exchange  the owner seeds the file to the other ranks in pieces of `piece_bytes` (async RCCL
            broadcasts over xGMI), overlapping the next round's fetch; the GPUs act as BitTorrent
            peers for each other (BASELINE configs 2 and 3)
  verify    every receiver hashes each received file on its own device with the owner's chunk
            boundaries (BLAKE3 per chunk + Merkle) and compares with the published Xet file hash --
            no CDC pass, and no trust in the owner: wrong boundaries or bytes give another hash

Elastic re-shard: a fetch that fails on its owner is reassigned to a rank that has not
tried that file yet (least queued bytes); an owner that fails twice is dropped from ownership and
its queued files move to the others.  Every rank derives the same plan from the all-gathered round
results, so the collective never diverges.  Only when every owner failed a file do all ranks raise
SwarmPullError together (no hang).  Reference counterpart: none (the reference stops at files on
disk; its only failure handling is the per-term waterfall, CONTRIBUTING.md:92-99).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist

from .. import _core, ops
from .. import device as zdev
from .swarm_load import assign_owners


class SwarmPullError(RuntimeError):
    pass


def _listing(repo, revision, repo_type, group, rank):
    """Rank 0 asks the hub once; every rank gets the same (commit, files)."""
    obj = [None]
    if rank == 0:
        try:
            obj[0] = ("ok", _core.list_repo_files(repo, revision, repo_type))
        except Exception as e:  # every rank must leave the collective the same way
            obj[0] = ("err", f"{type(e).__name__}: {e}")
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=group)
    status, val = obj[0]
    if status != "ok":
        raise SwarmPullError(f"listing {repo}@{revision} failed on rank 0: {val}")
    return val


def _all_ok(ok: bool, device, group) -> bool:
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    return int(flag.item()) == 0


def verify_with_lens(buf: torch.Tensor, lens: bytes, xet_hash: str) -> bool:
    """Xet file hash of `buf` with the given uint32 chunk sizes (BLAKE3 + Merkle on buf's device)."""
    n = buf.numel()
    if n == 0:
        return _core.xet_hex(_core.file_hash([])) == xet_hash
    if buf.device.type != "cuda":
        h = _core.xet_file_hash_lens(buf.numpy(), lens)
        return bool(h) and _core.xet_hex(h) == xet_hash
    sizes = np.frombuffer(lens, dtype=np.uint32)
    if int(sizes.sum(dtype=np.uint64)) != n or (len(sizes) and int(sizes.max()) > 128 * 1024):
        return False
    starts = np.concatenate([[0], np.cumsum(sizes, dtype=np.uint64)[:-1]]).astype(np.uint64)
    hashes = ops.hash_ranges(buf, starts, sizes)
    sz = torch.from_numpy(sizes.astype(np.int64)).to(buf.device)
    root = ops.merkle_roots(hashes, sz, [(0, len(sizes))], file_hash=True)
    return _core.xet_hex(root[0].cpu().numpy().tobytes()) == xet_hash


def swarm_pull(repo: str, revision: str = "main", group=None, device=None, *, p2p: bool = True, peers=None,
               tracker=None, dht: bool = True, dht_bootstrap=None, repo_type: str = "model",
               verify_received: bool = True, staging_bytes: int = 1 << 30, threads: int = 16,
               piece_bytes: int = 256 << 20, stats: dict | None = None) -> dict[str, torch.Tensor]:
    """Collective over `group`: returns {tensor_name: tensor} on this rank's device, every rank the
    full set.  `stats`, if given, is filled with this rank's byte counts (fetched / received) and the
    number of files reassigned after failed fetches."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
            else torch.device("cpu")
    device = torch.device(device)
    commit, files = _listing(repo, revision, repo_type, group, rank)
    st_files = [f for f in files if f["path"].endswith(".safetensors")]
    xet = [f for f in st_files if f["xet_hash"]]
    plain = [f for f in st_files if not f["xet_hash"]]
    todo = xet + plain
    bufs = [ops.padded_empty(f["size"], device)[: f["size"]] if device.type == "cuda"
            else torch.empty(f["size"], dtype=torch.uint8) for f in todo]
    # Ownership queues (identical on every rank): Xet files by LPT, largest first per owner; the
    # non-Xet safetensors (host pull) go to rank 0 as one item.
    owner = assign_owners([f["size"] for f in xet], world)
    queue: list[list] = [[] for _ in range(world)]
    for i in sorted(range(len(xet)), key=lambda i: (-xet[i]["size"], i)):
        queue[owner[i]].append(("xet", i))
    if plain:
        queue[0].append(("plain", tuple(range(len(xet), len(todo)))))
    granks = [dist.get_global_rank(group, r) for r in range(world)] if group is not None else list(range(world))
    fetcher = _Fetcher(repo, revision, repo_type, device, p2p, peers, tracker, dht, dht_bootstrap, staging_bytes,
                       threads)
    fault = os.environ.get("ZEST_SWARM_FAULT", "")  # "<rank>:<round>[,...]": that fetch raises (tests)
    faults = {tuple(int(x) for x in item.split(":")) for item in fault.split(",") if item}
    tried: dict = {}            # item -> ranks that failed it
    fails = [0] * world
    alive = [True] * world      # still an owner
    fetched_by: dict[int, int] = {}   # file index -> owner that fetched it
    lens_of: dict[int, bytes] = {}
    works, fetched_bytes, reassigned, j = [], 0, 0, 0
    while any(queue):
        this_round = [q.pop(0) if q else None for q in queue]
        item = this_round[rank]
        err, lens = "", []
        if item is not None:
            try:
                if (rank, j) in faults:
                    raise RuntimeError(f"injected fetch failure (round {j})")
                idx = [item[1]] if item[0] == "xet" else list(item[1])
                lens = fetcher.fetch([todo[i] for i in idx], [bufs[i] for i in idx])
            except Exception as e:  # reported through the all-gather: every rank replans the same way
                err = f"rank {rank}: {type(e).__name__}: {e}"
        meta = [None] * world
        dist.all_gather_object(meta, (err, lens), group=group)
        fatal = []
        for r, it in enumerate(this_round):
            if it is None:
                continue
            e, ls = meta[r]
            if e:
                fails[r] += 1
                tried.setdefault(it, set()).add(r)
                if fails[r] >= 2:   # a repeatedly failing owner: hand its queue to the others
                    alive[r] = False
                moves = [it] + (queue[r] if not alive[r] else [])
                if not alive[r]:
                    queue[r] = []
                for m in moves:
                    cands = [q for q in range(world) if alive[q] and q not in tried.get(m, set())]
                    if not cands:
                        fatal.append(e if m == it else f"no owner left for {m}")
                        continue
                    load = [sum(todo[x[1]]["size"] if x[0] == "xet" else 0 for x in queue[q]) for q in range(world)]
                    q = min(cands, key=lambda q: (load[q], q))
                    queue[q].append(m)
                    reassigned += 1
                continue
            idx = [it[1]] if it[0] == "xet" else list(it[1])
            for k, i in enumerate(idx):
                fetched_by[i] = r
                if ls and k < len(ls) and ls[k] is not None:
                    lens_of[i] = ls[k]
                if r == rank:
                    fetched_bytes += todo[i]["size"]
                # seed the file to every other rank, in pieces (async; overlaps the next round's fetch)
                n = todo[i]["size"]
                for off in range(0, n, piece_bytes):
                    works.append(dist.broadcast(bufs[i][off:off + min(piece_bytes, n - off)], granks[r], group=group,
                                                async_op=True))
        if fatal:
            for w in works:  # leave no collective of an earlier round in flight
                w.wait()
            raise SwarmPullError("; ".join(sorted(set(fatal))))
        j += 1
    for w in works:
        w.wait()
    bad = []
    if verify_received:
        for i, f in enumerate(todo):
            if fetched_by.get(i) == rank or not f["xet_hash"]:
                continue
            ok = verify_with_lens(bufs[i], lens_of[i], f["xet_hash"]) if i in lens_of \
                else zdev.xet_file_hash(bufs[i]) == f["xet_hash"]
            if not ok:
                bad.append(f["path"])
    if not _all_ok(not bad, device, group):
        raise zdev.VerifyError(f"rank {rank}: received files failed their Xet hash: {bad}" if bad
                               else f"rank {rank}: a peer rank received corrupt files")
    if stats is not None:
        stats.update(files=len(todo), owned=sum(1 for r in fetched_by.values() if r == rank),
                     fetched_bytes=fetched_bytes,
                     received_bytes=sum(f["size"] for i, f in enumerate(todo) if fetched_by.get(i) != rank),
                     reassigned=reassigned, rounds=j)
    out: dict[str, torch.Tensor] = {}
    for f, buf in zip(todo, bufs):
        if f["size"] == 0:
            continue
        hlen = int.from_bytes(buf[:8].cpu().numpy().tobytes(), "little")
        start, meta_ = zdev.parse_safetensors_header(buf[: 8 + hlen].cpu().numpy().tobytes())
        for k, v in zdev.tensor_views(buf, start, meta_).items():
            if k in out:
                raise ValueError(f"duplicate tensor {k} in {f['path']}")
            out[k] = v
    return out


class _Fetcher:
    """Fetches this rank's owned files into their buffers, one round at a time, and returns each
    file's chunk sizes (uint32 bytes; None for non-Xet files).  On a GPU the Xet files go
    device-direct through one DeviceXetPull; on CPU through one HostXetFetcher (in memory, no
    snapshot).  Both are built on first use and kept, so the hub session and the peer connections
    carry over between rounds.  Non-Xet safetensors come through the host pull."""

    def __init__(self, repo, revision, repo_type, device, p2p, peers, tracker, dht, dht_bootstrap, staging_bytes,
                 threads):
        self.repo, self.revision, self.repo_type, self.device = repo, revision, repo_type, device
        self.p2p, self.peers, self.tracker, self.dht = p2p, list(peers or []), tracker, dht
        self.dht_bootstrap, self.staging_bytes, self.threads = list(dht_bootstrap or []), staging_bytes, threads
        self._dp = None
        self._hf = None

    def fetch(self, files, bufs) -> list:
        lens: list = [None] * len(files)
        xet = [k for k, f in enumerate(files) if f["xet_hash"]]
        host = [k for k, f in enumerate(files) if not f["xet_hash"]]
        req = [(files[k]["xet_hash"], bufs[k].data_ptr(), files[k]["size"]) for k in xet]
        if xet and self.device.type == "cuda":
            if self._dp is None:
                self._dp = ops.hip().DeviceXetPull(self.repo, self.revision, self.repo_type, self.p2p, self.peers,
                                                   self.tracker, self.dht, self.dht_bootstrap,
                                                   self.device.index or 0, self.staging_bytes, self.threads)
            # the buffers exist (allocated on the current stream) before the pull's private stream
            # writes them; a device-wide sync would also wait for the previous rounds' RCCL broadcasts
            torch.cuda.current_stream(self.device).synchronize()
            res = self._dp.pull_files(req)
        elif xet:
            if self._hf is None:
                self._hf = _core.HostXetFetcher(self.repo, self.revision, self.repo_type, self.p2p, self.peers,
                                                self.tracker, self.dht, self.dht_bootstrap, self.threads)
            res = self._hf.fetch_files(req)
        else:
            res = []
        for k, r in zip(xet, res):
            lens[k] = r["chunk_lens"]
        if host:
            r = _core.pull(self.repo, self.revision, self.p2p, self.peers, self.tracker, self.dht,
                           self.dht_bootstrap, [files[k]["path"] for k in host], True, 0, self.repo_type)
            if r["failed_files"]:
                raise SwarmPullError(f"host pull failed for {r['failed_files']} file(s)")
            for k in host:
                bufs[k].copy_(zdev.load_file(os.path.join(r["snapshot_dir"], files[k]["path"]),
                                             self.device).view(torch.uint8))
        return lens
