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
        ser = world.chunk_clen.astype(np.uint64) + np.uint64(8)  # stored size (BG4-LZ4 frames in bf16 worlds)
        out_off = (np.cumsum(ser) - ser).astype(np.uint64)
        self.nbytes = int(ser.sum())
        self.buf = ops.padded_empty(self.nbytes, dev)
        for a in range(0, world.n_chunks, batch_chunks):
            b = min(world.n_chunks, a + batch_chunks)
            world.pack_serialized(content, a, b, self.buf, out_off[a:b])
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


class HbmCacheArena:
    """Warm seeding: every run of the local xorb disk cache (`{hex}` / `{hex}.{chunk_offset}`)
    uploaded once into one HBM buffer (restore the arena from the disk cache at serve
    start)."""

    def __init__(self, device="cuda:0", max_bytes: int | None = None):
        import json
        import os

        import numpy as np

        cfg = json.loads(_core.config_json())
        root = cfg["xorb_cache_dir"]
        runs = []
        total = 0
        for pfx in sorted(os.listdir(root)) if os.path.isdir(root) else []:
            d = os.path.join(root, pfx)
            if len(pfx) != 2 or not os.path.isdir(d):
                continue
            for name in sorted(os.listdir(d)):
                hx, _, off = name.partition(".")
                if len(hx) != 64 or (off and not off.isdigit()):
                    continue
                path = os.path.join(d, name)
                size = os.path.getsize(path)
                if max_bytes is not None and total + size > max_bytes:
                    break
                runs.append((hx, int(off or 0), path, size))
                total += size
        dev = torch.device(device)
        self.nbytes = total
        self.buf = ops.padded_empty(max(total, 1), dev)
        self.runs = []  # (hex, dev_off, chunk_ends, first_chunk)
        pos = 0
        for hx, first, path, size in runs:
            data = np.fromfile(path, dtype=np.uint8)
            try:
                idx = _core.index_chunks(data)
            except Exception:
                continue  # not a chunk run (corrupt file): skip
            if not idx:
                continue
            ends = [e[0] + 8 + e[1] for e in idx]
            n = ends[-1]
            self.buf[pos:pos + n].copy_(torch.from_numpy(data[:n]), non_blocking=False)
            self.runs.append((hx, pos, ends, first))
            pos += n
        self.used = pos


class HbmCacheSeedServer:
    """BEP XET seeder over an HbmCacheArena (falls back to the disk cache for anything else)."""

    def __init__(self, arena: HbmCacheArena, port: int = 0):
        H = ops.hip()
        dev = arena.buf.device
        self.arena = arena
        self.seeder = H.HbmSeeder(arena.buf.data_ptr(), max(arena.used, 1), dev.index or 0, port, True)
        for hx, off, ends, first in arena.runs:
            self.seeder.add_xorb(hx, int(off), ends, int(first))
        self.seeder.start()

    @property
    def port(self) -> int:
        return self.seeder.port

    def stats(self) -> dict:
        return self.seeder.stats()

    def stop(self) -> None:
        self.seeder.stop()


def main(argv=None) -> int:
    """`python -m zest_amd.seed [--port P] [--device cuda:0] [--max-gb G]`: seed the local xorb cache
    from HBM until interrupted."""
    import argparse
    import signal
    import threading

    ap = argparse.ArgumentParser(description="seed the local xorb cache from GPU memory")
    ap.add_argument("--port", type=int, default=6881)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--max-gb", "--hbm-cache-gb", dest="max_gb", type=float, default=None)
    a = ap.parse_args(argv)
    arena = HbmCacheArena(a.device, None if a.max_gb is None else int(a.max_gb * 1e9))
    srv = HbmCacheSeedServer(arena, a.port)
    print(f"HBM seeder: {len(arena.runs)} cached runs, {arena.used / 1e9:.2f} GB on {a.device}, "
          f"BT listen port {srv.port}", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    stop.wait()
    srv.stop()
    print("stats:", srv.stats(), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
