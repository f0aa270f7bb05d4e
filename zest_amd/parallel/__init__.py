"""Intra-node parallelism: one process per GPU, RCCL over xGMI via torch.distributed ("nccl").

* `exchange.RoundExchange`: per-round replication of arena regions over xGMI (RCCL p2p / coalesced
  broadcasts / slab all-gather, or peer-mapped HIP VMM arenas read by DMA copies or the K8 kernel),
  autotuned per machine; `map_peer_arenas` builds the peer mappings.
* `DevicePuller` (zest_amd.engine): owner-sharded term ingest from a pinned origin + that exchange —
  the swarm pull bench.py measures.
* `swarm_pull`: the same machinery fed by the network (public `pull(device="all")`): byte-balanced
  term shares fetched device-direct, rounds exchanged over xGMI, every chunk re-hashed on every GPU,
  Merkle-checked per file; survives a lost rank.
* `swarm_load`: replicate a pulled snapshot into every GPU's HBM, each file read by one owner rank.
* `init_from_env`: torchrun-style rendezvous (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*).
* `bind_local_numa`: pin a rank to the CPUs of its GPU's NUMA node, so its pinned host staging and
  origin pages are first-touched next to the GPU's PCIe root (8 ranks x ~57 GB/s of H2D must not
  cross the socket interconnect).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .swarm_load import assign_owners, swarm_load
from .swarm_pull import SwarmPullError, swarm_pull


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
        bind_local_numa(dev)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        import datetime
        kw = {"device_id": dev, "pg_options": nccl_options()} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, local, dev


def nccl_options():
    """ProcessGroupNCCL options for the swarm: RCCL's internal stream at high priority, so the piece
    exchange's kernels are dispatched ahead of the receive-side BLAKE3 verification that runs
    concurrently on a normal-priority stream (both want every CU; the exchange is on the critical
    path, the verification is not)."""
    from torch.distributed import ProcessGroupNCCL

    return ProcessGroupNCCL.Options(is_high_priority_stream=True)


def parse_cpulist(text: str) -> set[int]:
    """Linux cpulist syntax ("0-3,8,10-11") -> set of CPU ids."""
    cpus: set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_local_cpus(device, sysfs: str = "/sys/bus/pci/devices") -> set[int]:
    """CPUs on the NUMA node of `device`'s PCIe function (empty when sysfs does not say)."""
    p = torch.cuda.get_device_properties(device)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    try:
        with open(os.path.join(sysfs, bdf, "local_cpulist")) as f:
            return parse_cpulist(f.read())
    except (OSError, ValueError):
        return set()


def bind_local_numa(device, local_cpus: set[int] | None = None) -> list[int]:
    """Restrict this process to the CPUs near `device` (intersected with its current affinity).

    Call before allocating pinned host memory. Returns the CPUs bound to ([] = left unchanged:
    ZEST_NUMA_BIND=0, no sysfs information, or no overlap with the allowed CPU set)."""
    if os.environ.get("ZEST_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return []
    near = gpu_local_cpus(device) if local_cpus is None else local_cpus
    allowed = os.sched_getaffinity(0)
    both = sorted(near & allowed)
    if not both or set(both) == allowed:
        return []
    os.sched_setaffinity(0, both)
    return both


def __getattr__(name):
    if name == "DevicePuller":
        from ..engine import DevicePuller
        return DevicePuller
    raise AttributeError(name)


__all__ = ["DevicePuller", "assign_owners", "bind_local_numa", "gpu_local_cpus", "init_from_env", "nccl_options",
           "parse_cpulist", "swarm_load", "swarm_pull", "SwarmPullError"]
