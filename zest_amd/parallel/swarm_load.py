"""Intra-node swarm load of a pulled snapshot: every GPU ends up with every tensor in its HBM, but
each file is read from disk and pushed over PCIe by exactly one rank; the other ranks receive it
over xGMI (RCCL broadcast from the owner, i.e. GPUs acting as seeders for each other).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm; "gloo" on CPU for tests).
Owner assignment is a longest-processing-time greedy split by file size, so disk + PCIe work is
balanced.  With `xet_hashes`, the owner verifies each file on its GPU before seeding it (receivers
can re-verify with `verify_all=True`), so a corrupt disk cache never propagates.

Reference counterpart: none (the reference stops at files on disk); this is SURVEY §2.E P1/P7 and
§2.F applied to the load step.
"""
from __future__ import annotations

import os
import struct

import torch
import torch.distributed as dist

from .. import device as zdev
from .. import ops


def assign_owners(sizes: list[int], world: int) -> list[int]:
    """LPT greedy: largest file to the least-loaded rank.  Deterministic on every rank."""
    load = [0] * world
    owner = [0] * len(sizes)
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[i] = r
        load[r] += sizes[i]
    return owner


def swarm_load(snapshot_dir: str, group=None, device=None, xet_hashes: dict[str, str] | None = None,
               files: list[str] | None = None, verify_all: bool = False) -> dict[str, torch.Tensor]:
    """Collective: call on every rank of `group`. Returns {tensor_name: tensor} on this rank's device."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
            else torch.device("cpu")
    device = torch.device(device)
    if files is None:
        files = sorted(str(p.relative_to(snapshot_dir)) for p in zdev._rglob(snapshot_dir)
                       if p.name.endswith(".safetensors"))
    sizes = [os.path.getsize(os.path.join(snapshot_dir, f)) for f in files]
    # Every rank must agree on the file list and sizes (same snapshot on shared or replicated disk).
    sig = torch.tensor([len(files), sum(sizes)], dtype=torch.int64, device=device)
    ref = sig.clone()
    dist.broadcast(ref, 0, group=group)
    if not torch.equal(sig, ref):
        raise RuntimeError(f"rank {rank}: snapshot differs from rank 0 ({sig.tolist()} vs {ref.tolist()})")
    owner = assign_owners(sizes, world)
    bufs = []
    for i, rel in enumerate(files):
        if owner[i] == rank:
            buf = zdev.load_file(os.path.join(snapshot_dir, rel), device)
            if xet_hashes and rel in xet_hashes:
                got = zdev.xet_file_hash(buf)
                if got != xet_hashes[rel]:
                    raise zdev.VerifyError(f"rank {rank}: {rel} hash {got} != {xet_hashes[rel]}")
        else:
            buf = ops.padded_empty(sizes[i], device)[:sizes[i]] if device.type == "cuda" \
                else torch.empty(sizes[i], dtype=torch.uint8)
        bufs.append(buf)
    global_ranks = [dist.get_global_rank(group, r) for r in range(world)] if group is not None else list(range(world))
    works = [dist.broadcast(bufs[i], global_ranks[owner[i]], group=group, async_op=True)
             for i in range(len(files)) if sizes[i] > 0]
    for w in works:
        w.wait()
    out: dict[str, torch.Tensor] = {}
    for i, rel in enumerate(files):
        buf = bufs[i]
        if verify_all and xet_hashes and rel in xet_hashes and owner[i] != rank:
            got = zdev.xet_file_hash(buf)
            if got != xet_hashes[rel]:
                raise zdev.VerifyError(f"rank {rank}: received {rel} hash {got} != {xet_hashes[rel]}")
        (hlen,) = struct.unpack("<Q", buf[:8].cpu().numpy().tobytes())
        start, meta = zdev.parse_safetensors_header(buf[:8 + hlen].cpu().numpy().tobytes())
        for k, v in zdev.tensor_views(buf, start, meta).items():
            out[k] = v
    return out
