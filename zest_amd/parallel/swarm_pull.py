"""Intra-node swarm pull: every GPU of a node ends up with every tensor of a repository in its HBM,
while each Xet file crosses the network (peers / CDN / local xorb cache) exactly once.

    # one process per GPU (torchrun), backend "nccl" = RCCL over xGMI
    tensors = swarm_pull("meta-llama/Llama-3.1-70B")   # collective; every rank gets all tensors

Each Xet-backed safetensors file has one owner rank (LPT split by size, as `zest pull --gpus N`
assigns files).  The pull runs in rounds of one owned file per rank; a round's broadcasts overlap
the next round's network fetch.  The owner pulls it device-direct (`_hip.DeviceXetPull`: compressed runs -> pinned
staging -> GPU decode + BLAKE3 + Merkle check, with the peer-quarantine / CDN-repair rules of the
native bridge) and then seeds it to the other GPUs with an RCCL broadcast over xGMI -- the GPUs act
as BitTorrent peers for each other, with broadcast as the piece exchange (BASELINE configs 2 and 3,
SURVEY §3.6).  Receivers re-derive the file's Xet hash on their own GPU before handing out tensors,
so no rank trusts another rank's bytes.  Non-Xet safetensors files are fetched by rank 0 through
the host pull and broadcast the same way.

On CPU process groups (gloo) the owner fetches through the host pull instead and loads the file;
the exchange and the receive-side verification are the same, which is what the multi-process CPU
tests exercise.  Reference counterpart: none (the reference stops at files on disk).
"""
from __future__ import annotations

import os

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


def swarm_pull(repo: str, revision: str = "main", group=None, device=None, *, p2p: bool = True, peers=None,
               tracker=None, dht: bool = True, dht_bootstrap=None, repo_type: str = "model",
               verify_received: bool = True, staging_bytes: int = 1 << 30, threads: int = 16,
               stats: dict | None = None) -> dict[str, torch.Tensor]:
    """Collective over `group`: returns {tensor_name: tensor} on this rank's device, every rank the
    full set.  `stats`, if given, is filled with this rank's byte counts (fetched / received)."""
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
    owner = assign_owners([f["size"] for f in xet], world) + [0] * len(plain)
    todo = xet + plain
    mine = [i for i, o in enumerate(owner) if o == rank]
    bufs = [ops.padded_empty(f["size"], device)[: f["size"]] if device.type == "cuda"
            else torch.empty(f["size"], dtype=torch.uint8) for f in todo]
    # Rounds: round j is every rank's j-th owned Xet file (rank 0's non-Xet files, fetched through
    # the host pull, form its last round).  A round's broadcasts are issued
    # asynchronously, so they cross xGMI while the owners fetch the next round's files from the
    # network: the pull takes ~max(network, xGMI) instead of their sum.
    plan = [[[i] for i in range(len(xet)) if owner[i] == r] for r in range(world)]
    if plain:
        plan[0].append(list(range(len(xet), len(todo))))
    n_rounds = max(len(p) for p in plan)
    granks = [dist.get_global_rank(group, r) for r in range(world)] if group is not None else list(range(world))
    fetcher = _Fetcher(repo, revision, repo_type, device, p2p, peers, tracker, dht, dht_bootstrap, staging_bytes,
                       threads)
    works = []
    for j in range(n_rounds):
        err = ""
        mine_j = plan[rank][j] if j < len(plan[rank]) else []
        try:
            fetcher.fetch([todo[i] for i in mine_j], [bufs[i] for i in mine_j])
        except Exception as e:  # reported after the all-reduce, so no rank is left waiting in a broadcast
            err = f"rank {rank}: {type(e).__name__}: {e}"
        if not _all_ok(not err, device, group):
            for w in works:  # leave no collective of an earlier round in flight
                w.wait()
            raise SwarmPullError(err or f"rank {rank}: a peer rank failed to fetch its files")
        for r in range(world):
            for i in (plan[r][j] if j < len(plan[r]) else []):
                if todo[i]["size"] > 0:
                    works.append(dist.broadcast(bufs[i], granks[r], group=group, async_op=True))
    for w in works:
        w.wait()
    bad = []
    if verify_received:
        for i, f in enumerate(todo):
            if owner[i] != rank and f["xet_hash"] and zdev.xet_file_hash(bufs[i]) != f["xet_hash"]:
                bad.append(f["path"])
    if not _all_ok(not bad, device, group):
        raise zdev.VerifyError(f"rank {rank}: received files failed their Xet hash: {bad}" if bad
                               else f"rank {rank}: a peer rank received corrupt files")
    if stats is not None:
        stats.update(files=len(todo), owned=len(mine), fetched_bytes=sum(todo[i]["size"] for i in mine),
                     received_bytes=sum(f["size"] for i, f in enumerate(todo) if owner[i] != rank))
    out: dict[str, torch.Tensor] = {}
    for f, buf in zip(todo, bufs):
        if f["size"] == 0:
            continue
        hlen = int.from_bytes(buf[:8].cpu().numpy().tobytes(), "little")
        start, meta = zdev.parse_safetensors_header(buf[: 8 + hlen].cpu().numpy().tobytes())
        for k, v in zdev.tensor_views(buf, start, meta).items():
            if k in out:
                raise ValueError(f"duplicate tensor {k} in {f['path']}")
            out[k] = v
    return out


class _Fetcher:
    """Fetches this rank's owned files into their buffers, one round at a time.  On a GPU the Xet
    files go device-direct through one DeviceXetPull (built on first use and kept, so the hub
    session and the peer connections carry over between rounds); otherwise, and for non-Xet
    files, through the host pull."""

    def __init__(self, repo, revision, repo_type, device, p2p, peers, tracker, dht, dht_bootstrap, staging_bytes,
                 threads):
        self.repo, self.revision, self.repo_type, self.device = repo, revision, repo_type, device
        self.p2p, self.peers, self.tracker, self.dht = p2p, list(peers or []), tracker, dht
        self.dht_bootstrap, self.staging_bytes, self.threads = list(dht_bootstrap or []), staging_bytes, threads
        self._dp = None

    def fetch(self, files, bufs):
        if not files:
            return
        xet = [(f, b) for f, b in zip(files, bufs) if f["xet_hash"]]
        host = [(f, b) for f, b in zip(files, bufs) if not f["xet_hash"]]
        if self.device.type == "cuda" and xet:
            if self._dp is None:
                self._dp = ops.hip().DeviceXetPull(self.repo, self.revision, self.repo_type, self.p2p, self.peers,
                                                   self.tracker, self.dht, self.dht_bootstrap,
                                                   self.device.index or 0, self.staging_bytes, self.threads)
            torch.cuda.synchronize(self.device)  # the buffers exist before the pull's private stream writes them
            self._dp.pull_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in xet])
        else:
            host = xet + host
        if host:
            r = _core.pull(self.repo, self.revision, self.p2p, self.peers, self.tracker, self.dht,
                           self.dht_bootstrap, [f["path"] for f, _ in host], True, 0, self.repo_type)
            if r["failed_files"]:
                raise SwarmPullError(f"host pull failed for {r['failed_files']} file(s)")
            for f, b in host:
                b.copy_(zdev.load_file(os.path.join(r["snapshot_dir"], f["path"]), self.device).view(torch.uint8))
