"""Seed mode from HBM: serve a model's xorbs to BitTorrent (BEP XET) peers straight out of GPU memory.

`HbmXorbArena` serializes every xorb of a model (8-byte chunk headers + payloads, the CAS wire
form) into one device buffer with the GPU pack kernel (K7); `HbmSeedServer` registers each xorb's
chunk boundaries with the native `_hip.HbmSeeder`, whose provider copies requested chunk runs
HBM → pinned host → socket with no intermediate host copy.  This is the MI355X counterpart of the
reference's disk-backed seeding (src/server.zig:187-215) sized for 288 GB of HBM per GPU
(BASELINE config: "Mixtral-8x7B seed mode: serve xorbs from 288 GB HBM, measure chunks_served/s").
"""
from __future__ import annotations

import numpy as np
import torch

from . import _core, ops
from .synthetic import SyntheticWorld


class HbmXorbArena:
    def __init__(self, world: SyntheticWorld, content: torch.Tensor, device=None, batch_chunks: int = 1 << 20):
        if world.terms is None:
            raise ValueError("world must be built (build_on_device / build_on_host) first")
        self.world = world
        dev = torch.device(device) if device is not None else content.device
        ser = world.chunk_len.astype(np.uint64) + np.uint64(8)
        out_off = (np.cumsum(ser) - ser).astype(np.uint64)
        self.nbytes = int(ser.sum())
        self.buf = ops.padded_empty(self.nbytes, dev)
        for a in range(0, world.n_chunks, batch_chunks):
            b = min(world.n_chunks, a + batch_chunks)
            ops.pack_chunks(content, world.chunk_off[a:b], world.chunk_len[a:b], out_off[a:b], self.buf)
        x0 = world.xorb_chunk0
        x1 = np.concatenate([x0[1:], [world.n_chunks]])
        self.xorb_off = out_off[x0]
        cum = np.cumsum(ser)
        self.xorb_ends = [(cum[a:b] - (cum[a] - ser[a])).astype(np.uint64) for a, b in zip(x0, x1)]
        # xorb hashes on the GPU (Merkle over each xorb's chunk hashes, K2)
        hashes = torch.from_numpy(np.ascontiguousarray(world.chunk_hashes)).to(dev)
        sizes = torch.from_numpy(world.chunk_len.astype(np.int64)).to(dev)
        roots = ops.merkle_roots(hashes, sizes, [(int(a), int(b - a)) for a, b in zip(x0, x1)], file_hash=False)
        self.xorb_hashes = [bytes(r) for r in roots.cpu().numpy()]
        self.xorb_hex = [_core.xet_hex(h) for h in self.xorb_hashes]
        torch.cuda.synchronize(dev) if dev.type == "cuda" else None


class HbmSeedServer:
    """BEP XET listener backed by an HbmXorbArena (optionally falling back to the disk cache)."""

    def __init__(self, arena: HbmXorbArena, port: int = 0, disk_fallback: bool = False):
        from . import ops as _ops
        H = _ops.hip()
        dev = arena.buf.device
        self.arena = arena
        self.seeder = H.HbmSeeder(arena.buf.data_ptr(), arena.nbytes, dev.index or 0, port, disk_fallback)
        for hx, off, ends in zip(arena.xorb_hex, arena.xorb_off, arena.xorb_ends):
            self.seeder.add_xorb(hx, int(off), ends.tolist())
        self.seeder.start()

    @property
    def port(self) -> int:
        return self.seeder.port

    def stats(self) -> dict:
        return self.seeder.stats()

    def stop(self) -> None:
        self.seeder.stop()
