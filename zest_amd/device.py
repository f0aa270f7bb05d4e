"""Snapshot → HBM: stream safetensors files into device memory, verify them on the GPU against
their Xet file hashes, and hand back tensor views (no host copy of the model is kept).

This is the `zest.pull(..., device=...)` path of the north star: the reference stops at files on
disk (python/zest/client.py:32-46); here `from_pretrained`-style consumers get weights already
resident in HBM.  Verification re-derives the Xet file hash from the bytes that actually landed
in device memory: GPU CDC candidates (K5) → Xet min/max selection → BLAKE3 keyed chunk hashes (K1)
→ Merkle tree + file hash (K2), compared with the hub's `xetHash`.

File bytes are streamed through two pinned host staging buffers on a side HIP stream, so disk
reads overlap PCIe transfers.
"""
from __future__ import annotations

import json
import os
import struct
from dataclasses import dataclass

import numpy as np
import torch

from . import _core, ops

ST_DTYPES = {
    "BF16": torch.bfloat16, "F16": torch.float16, "F32": torch.float32, "F64": torch.float64,
    "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
    "BOOL": torch.bool, "F8_E4M3": torch.float8_e4m3fn, "F8_E5M2": torch.float8_e5m2,
}
for _name, _attr in (("U16", "uint16"), ("U32", "uint32"), ("U64", "uint64")):
    if hasattr(torch, _attr):
        ST_DTYPES[_name] = getattr(torch, _attr)


class VerifyError(RuntimeError):
    pass


def parse_safetensors_header(head: bytes) -> tuple[int, dict]:
    """Returns (data_start, metadata) from the first bytes of a .safetensors file."""
    if len(head) < 8:
        raise ValueError("not a safetensors file (short)")
    (hlen,) = struct.unpack("<Q", head[:8])
    if hlen > 100 << 20:
        raise ValueError("safetensors header too large")
    if len(head) < 8 + hlen:
        raise ValueError("need more header bytes")
    meta = json.loads(head[8:8 + hlen])
    return 8 + hlen, meta


def read_safetensors_header(path: str) -> tuple[int, dict]:
    with open(path, "rb") as f:
        (hlen,) = struct.unpack("<Q", f.read(8))
        return parse_safetensors_header(struct.pack("<Q", hlen) + f.read(hlen))


def tensor_views(buf: torch.Tensor, data_start: int, meta: dict) -> dict[str, torch.Tensor]:
    """Typed views into a uint8 buffer holding one whole safetensors file."""
    out = {}
    for name, ent in meta.items():
        if name == "__metadata__":
            continue
        dt = ST_DTYPES.get(ent["dtype"])
        if dt is None:
            raise ValueError(f"{name}: unsupported dtype {ent['dtype']}")
        a, b = ent["data_offsets"]
        raw = buf[data_start + a:data_start + b]
        esz = torch.empty((), dtype=dt).element_size()
        if (data_start + a) % esz:  # misaligned entry (hand-written files): copy out
            raw = raw.clone()
        t = raw.view(dt) if b > a else torch.empty(0, dtype=dt, device=buf.device)
        out[name] = t.view(ent["shape"]) if ent["shape"] else t.reshape(())
    return out


def load_file(path: str, device, staging_bytes: int = 64 << 20) -> torch.Tensor:
    """Read a whole file into a padded uint8 tensor on `device`."""
    device = torch.device(device)
    size = os.path.getsize(path)
    if device.type != "cuda":
        buf = torch.empty(size, dtype=torch.uint8)
        with open(path, "rb") as f:
            f.readinto(memoryview(buf.numpy()))
        return buf
    dst = ops.padded_empty(size, device)
    if size == 0:
        return dst[:0]
    stage = [torch.empty(staging_bytes, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    done = [None, None]
    stream = torch.cuda.Stream(device=device)
    off, k = 0, 0
    with open(path, "rb", buffering=0) as f:
        while off < size:
            slot = k & 1
            if done[slot] is not None:
                done[slot].synchronize()
            n = min(staging_bytes, size - off)
            mv = memoryview(stage[slot].numpy())[:n]
            got = 0
            while got < n:
                r = f.readinto(mv[got:])
                if not r:
                    raise IOError(f"{path}: short read at {off + got}")
                got += r
            with torch.cuda.stream(stream):
                dst[off:off + n].copy_(stage[slot][:n], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
            done[slot] = ev
            off += n
            k += 1
    torch.cuda.current_stream(device).wait_stream(stream)
    stream.synchronize()
    return dst[:size]


def xet_file_hash(buf: torch.Tensor) -> str:
    """Xet file hash (xet hex) of a uint8 buffer; runs entirely on the GPU for cuda tensors."""
    n = buf.numel()
    if n == 0:
        return _core.xet_hex(_core.file_hash([]))
    if buf.device.type != "cuda":
        return _core.xet_hex(_core.xet_file_hash(buf.numpy()))
    cands = ops.cdc_candidates(buf)
    ends = ops.select_chunks(cands, n)
    starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)
    lens = (ends - starts).astype(np.uint32)
    hashes = ops.hash_ranges(buf, starts, lens)
    sizes = torch.from_numpy(lens.astype(np.int64)).to(buf.device)
    root = ops.merkle_roots(hashes, sizes, [(0, len(lens))], file_hash=True)
    return _core.xet_hex(root[0].cpu().numpy().tobytes())


@dataclass
class LoadedFile:
    path: str
    buffer: torch.Tensor
    tensors: dict
    verified: bool


def load_snapshot(snapshot_dir: str, device="cuda:0", xet_hashes: dict[str, str] | None = None,
                  files: list[str] | None = None) -> dict[str, torch.Tensor]:
    """Load every *.safetensors file of a snapshot onto `device`; verify against `xet_hashes`
    (path → xet hex) when given.  Returns {tensor_name: tensor}."""
    loaded = load_snapshot_files(snapshot_dir, device, xet_hashes, files)
    out: dict[str, torch.Tensor] = {}
    for lf in loaded:
        for k, v in lf.tensors.items():
            if k in out:
                raise ValueError(f"duplicate tensor {k} in {lf.path}")
            out[k] = v
    return out


def load_snapshot_files(snapshot_dir, device="cuda:0", xet_hashes=None, files=None) -> list[LoadedFile]:
    if files is None:
        files = sorted(str(p.relative_to(snapshot_dir)) for p in _rglob(snapshot_dir) if p.name.endswith(".safetensors"))
    out = []
    for rel in files:
        path = os.path.join(snapshot_dir, rel)
        buf = load_file(path, device)
        verified = False
        if xet_hashes and rel in xet_hashes:
            got = xet_file_hash(buf)
            if got != xet_hashes[rel]:
                raise VerifyError(f"{rel}: device bytes hash {got} != hub xetHash {xet_hashes[rel]}")
            verified = True
        head = buf[:min(buf.numel(), 8)].cpu().numpy().tobytes()
        (hlen,) = struct.unpack("<Q", head)
        start, meta = parse_safetensors_header(buf[:8 + hlen].cpu().numpy().tobytes())
        out.append(LoadedFile(rel, buf, tensor_views(buf, start, meta), verified))
    return out


def _rglob(root):
    from pathlib import Path
    return Path(root).rglob("*")
