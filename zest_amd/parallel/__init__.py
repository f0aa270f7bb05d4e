"""Intra-node parallelism: one process per GPU, RCCL over xGMI via torch.distributed ("nccl").

* `DevicePuller` (zest_amd.engine): owner-sharded term ingest + peer-to-peer round exchange of the
  HBM arena — the swarm pull used by bench.py.
* `swarm_load`: replicate a pulled snapshot into every GPU's HBM, each file read by one owner rank.
* `init_from_env`: torchrun-style rendezvous (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .swarm_load import assign_owners, swarm_load


def init_from_env(backend: str | None = None, timeout_s: int = 600):
    """Initialise torch.distributed from torchrun env vars; returns (rank, world, local_rank, device).

    A single process without RANK set runs as world size 1 without a process group."""
    if "RANK" not in os.environ or "WORLD_SIZE" not in os.environ:
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        return 0, 1, 0, dev
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        import datetime
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, local, dev


def __getattr__(name):
    if name == "DevicePuller":
        from ..engine import DevicePuller
        return DevicePuller
    raise AttributeError(name)


__all__ = ["DevicePuller", "assign_owners", "init_from_env", "swarm_load"]
