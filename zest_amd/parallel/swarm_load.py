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


def _agree(ok: bool, device, group) -> bool:
    """True on every rank iff `ok` on every rank."""
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    return int(flag.item()) == 0


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
    bufs = [None if owner[i] == rank else
            (ops.padded_empty(sizes[i], device)[:sizes[i]] if device.type == "cuda"
             else torch.empty(sizes[i], dtype=torch.uint8)) for i in range(len(files))]
    global_ranks = [dist.get_global_rank(group, r) for r in range(world)] if group is not None else list(range(world))
    # Rounds of one owned file per rank: round j's broadcasts cross xGMI while the owners read and
    # upload round j + 1's files.  A failed read or owner-side hash check is agreed on by every rank
    # (all-reduce) before any broadcast of that round, so no rank waits in a broadcast that its
    # owner will never send.
    plan = [[i for i in range(len(files)) if owner[i] == r] for r in range(world)]
    works = []
    for j in range(max(len(p) for p in plan)):
        err = ""
        if j < len(plan[rank]):
            i = plan[rank][j]
            rel = files[i]
            try:
                bufs[i] = zdev.load_file(os.path.join(snapshot_dir, rel), device)
                if xet_hashes and rel in xet_hashes:
                    got = zdev.xet_file_hash(bufs[i])
                    if got != xet_hashes[rel]:
                        err = f"rank {rank}: {rel} hash {got} != {xet_hashes[rel]}"
            except OSError as e:
                err = f"rank {rank}: reading {rel}: {e}"
        if not _agree(not err, device, group):
            for w in works:
                w.wait()
            raise zdev.VerifyError(err or f"rank {rank}: a peer rank could not load or verify its file")
        for r in range(world):
            if j < len(plan[r]) and sizes[plan[r][j]] > 0:
                works.append(dist.broadcast(bufs[plan[r][j]], global_ranks[r], group=group, async_op=True))
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
