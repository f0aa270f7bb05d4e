"""Synthetic Xet world: a model repository materialized as files -> CDC chunks -> xorbs -> terms.

This plays the role of HuggingFace's Xet storage for offline benchmarks and tests (there is no
network): it produces exactly what a Xet uploader would (CDC boundaries with the real gear table,
keyed-BLAKE3 chunk hashes, 64 MiB xorbs packed across files, per-file reconstruction terms,
Merkle file hashes) and the byte runs a CAS/CDN returns for each term's url_range
(`[8-byte chunk header | payload]*`).  Reference context: the reconstruction JSON consumed at
xet_bridge.zig:133-142 and parallel_download.zig:102-126 (terms + fetch_info url_range).

GPU path (`build_on_device`): content generation, CDC candidates, chunk hashes, Merkle file
hashes and xorb packing all run as HIP kernels (zest_amd.ops); the host only selects boundaries
over the sparse candidates and plans xorbs/terms (vectorized numpy + _core.plan_xorbs).
CPU path (`build_on_host`): the same plan from the C++ host core, for small models in tests.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

import numpy as np
import torch

from . import _core, models, ops

MAX_XORB_BYTES = 64 << 20
MAX_XORB_CHUNKS = 8192
FILE_ALIGN = 4096
MODES = {"random": 0, "bf16": 1}


def _file_seed(seed: int, idx: int) -> int:
    return int.from_bytes(hashlib.blake2b(f"{seed}:{idx}".encode(), digest_size=8).digest(), "little")


@dataclass
class FileEntry:
    path: str
    size: int
    arena_off: int
    header: bytes          # safetensors header bytes (b"" for regular files)
    data_seed: int
    xet: bool              # Xet-backed (weights) vs regular small file
    content: bytes = b""   # for regular (non-Xet) files


class SyntheticWorld:
    """Layout + Xet metadata of one synthetic repository."""

    def __init__(self, spec: models.ModelSpec | str, seed: int = 0, mode: str = "random",
                 revision_sha: str | None = None, max_xorb_bytes: int = MAX_XORB_BYTES, compression: str = "none"):
        """compression: "none" stores every chunk raw (what Xet does for random bytes); "bg4" compresses
        each chunk with BG4 + LZ4 on the GPU (build_on_device) and keeps the frame when it is smaller,
        as Xet does for bf16 checkpoints."""
        self.spec = models.get(spec) if isinstance(spec, str) else spec
        if compression not in ("none", "bg4"):
            raise ValueError("compression must be 'none' or 'bg4'")
        self.compression = compression
        self.max_xorb_bytes = max_xorb_bytes
        self.seed = seed
        self.mode = mode
        if mode not in MODES:
            raise ValueError(f"mode must be one of {list(MODES)}")
        self.shards = self.spec.shards()
        self.files: list[FileEntry] = []
        off = 0
        for i, sh in enumerate(self.shards):
            self.files.append(FileEntry(sh.path, sh.size, off, sh.header, _file_seed(seed, i), True))
            off = (off + sh.size + FILE_ALIGN - 1) // FILE_ALIGN * FILE_ALIGN
        self.arena_bytes = off
        for path, content in self.spec.small_files(self.shards).items():
            self.files.append(FileEntry(path, len(content), -1, b"", 0, False, content))
        self.commit = revision_sha or hashlib.sha1(f"{self.spec.repo_id}:{seed}:{mode}".encode()).hexdigest()
        self.xet_files = [f for f in self.files if f.xet]
        # filled by build_*
        self.chunk_off = None   # uint64 arena offset of each chunk (global arena order)
        self.chunk_len = None   # uint32
        self.chunk_file = None  # int32 file index (into xet_files)
        self.file_chunk0 = None  # first global chunk per xet file
        self.file_nchunks = None
        self.file_hashes = None  # uint8 [n_files, 32]
        self.chunk_hashes = None  # uint8 [n_chunks, 32] (host copy)
        self.xorb_of = None       # int64 per chunk
        self.ser_off = None       # uint64 offset of the chunk header inside its xorb
        self.terms = None         # structured array, see _plan_terms
        self.chunk_clen = None    # uint32 stored payload length (== chunk_len when raw)
        self.chunk_scheme = None  # uint8 0 = none, 2 = BG4-LZ4

    # ------------------------------------------------------------------------------------------
    @property
    def model_bytes(self) -> int:
        return sum(f.size for f in self.xet_files)

    @property
    def n_chunks(self) -> int:
        return 0 if self.chunk_len is None else len(self.chunk_len)

    def file_bytes_host(self, f: FileEntry) -> bytes:
        """Regenerate a file's bytes on the host (small models / tests)."""
        if not f.xet:
            return f.content
        data = np.empty(f.size - len(f.header), dtype=np.uint8)
        _host_fill(data, f.data_seed, MODES[self.mode])
        return f.header + data.tobytes()

    # ------------------------------------------------------------------------------------------
    # Device build (bench path)
    # ------------------------------------------------------------------------------------------
    def generate_on_device(self, arena: torch.Tensor) -> None:
        """Write every Xet file's bytes at its arena offset (header + synthetic weights)."""
        for f in self.xet_files:
            hdr = torch.frombuffer(bytearray(f.header), dtype=torch.uint8)
            arena[f.arena_off:f.arena_off + len(f.header)].copy_(hdr)
            data = arena[f.arena_off + len(f.header):f.arena_off + f.size]
            ops.fill_synthetic(data, f.data_seed, 0, MODES[self.mode])

    def build_on_device(self, arena: torch.Tensor, hash_batch: int = 1 << 20, shard=None, ser_store=None) -> None:
        """CDC + chunk hashes + file hashes (+ BG4-LZ4 stored sizes) + xorb/term plan, from content
        already in `arena`.

        shard = (rank, n_ranks, group): each rank chunks, hashes and compresses only the files it
        owns (byte-balanced LPT over the file sizes), then the per-file results (~49 B per chunk:
        offsets, sizes, hashes, stored sizes) are all-gathered, so every rank ends with the same plan
        at ~1/n of the GPU work (bench.py at N > 1; the content itself is regenerated on every rank,
        which is cheap).

        ser_store = (ptr, cap): pinned host memory that receives every chunk serialized the way the
        CAS serves it ([8-byte header | stored payload], chunk order) straight from this build's
        compression, so a one-rank origin (whose layout is exactly that: engine.DevicePuller, terms
        back to back) adopts the bytes instead of compressing every chunk a second time (compressed
        worlds only; unsharded builds only).  On return `self.serialized` = (ptr, cap, nbytes)."""
        nf = len(self.xet_files)
        self.serialized = None
        self._ser_sink = None
        if ser_store is not None and self.compression == "bg4" and (shard is None or shard[1] == 1):
            self._ser_sink = [int(ser_store[0]), int(ser_store[1]), 0, None]  # ptr, cap, written, tmp
        if shard is None:
            own = list(range(nf))
        else:
            from .parallel.swarm_load import assign_owners
            rank, n_ranks, group = shard
            owner = assign_owners([f.size for f in self.xet_files], n_ranks)
            own = [i for i in range(nf) if owner[i] == rank]
        per_file = {i: self._build_file(arena, i, hash_batch) for i in own}
        if shard is not None and shard[1] > 1:
            import torch.distributed as dist
            objs = [None] * shard[1]
            dist.all_gather_object(objs, per_file, group=shard[2])
            for o in objs:
                per_file.update(o)
        if self._ser_sink is not None:
            ptr, cap, n, _ = self._ser_sink
            self.serialized = (ptr, cap, n)
            self._ser_sink = None
        parts = [per_file[i] for i in range(nf)]
        self._set_chunks(np.concatenate([p["offs"] for p in parts]), np.concatenate([p["lens"] for p in parts]),
                         np.concatenate([np.full(len(p["lens"]), i, dtype=np.int32) for i, p in enumerate(parts)]))
        self.chunk_hashes = np.concatenate([p["hashes"] for p in parts])
        self.file_hashes = np.stack([p["file_hash"] for p in parts])
        if self.compression == "bg4":
            self.chunk_clen = np.concatenate([p["clen"] for p in parts])
            self.chunk_scheme = np.concatenate([p["scheme"] for p in parts])
        self._plan_xorbs()

    def _build_file(self, arena: torch.Tensor, i: int, hash_batch: int) -> dict:
        """One Xet file on the GPU: CDC boundaries (K5), chunk hashes (K1), file hash (K2) and, for
        compressed worlds, every chunk's BG4-LZ4 stored size and scheme (frames discarded: the
        origin build compresses its own share again)."""
        f = self.xet_files[i]
        region = arena[f.arena_off:f.arena_off + f.size]
        ends = ops.select_chunks(ops.cdc_candidates(region), f.size)
        starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)
        offs = starts + np.uint64(f.arena_off)
        lens = (ends - starts).astype(np.uint32)
        dev = arena.device
        hashes = torch.empty((len(lens), 32), dtype=torch.uint8, device=dev)
        for a in range(0, len(lens), hash_batch):
            b = min(len(lens), a + hash_batch)
            hashes[a:b] = ops.hash_ranges(arena, offs[a:b], lens[a:b])
        sizes = torch.from_numpy(lens.astype(np.int64)).to(dev)
        fh = ops.merkle_roots(hashes, sizes, [(0, len(lens))], file_hash=True)
        out = {"offs": offs, "lens": lens, "hashes": hashes.cpu().numpy(), "file_hash": fh[0].cpu().numpy()}
        if self.compression == "bg4":
            clen = lens.astype(np.uint32).copy()
            scheme = np.zeros(len(lens), dtype=np.uint8)
            for a in range(0, len(lens), 8192):
                b = min(len(lens), a + 8192)
                frames, flen = ops.compress_chunks(arena, offs[a:b], lens[a:b], bg4=True)
                keep = flen > 0
                clen[a:b][keep] = flen[keep]
                scheme[a:b][keep] = 2
                if self._ser_sink is not None:
                    self._sink_frames(arena, frames, offs[a:b], lens[a:b], clen[a:b], scheme[a:b])
                del frames
            out["clen"], out["scheme"] = clen, scheme
        return out

    def _sink_frames(self, arena, frames, offs, lens, clen, scheme) -> None:
        """Serialize one compressed batch ([header | frame or raw chunk] per chunk, compact) on the
        GPU and append it to the pinned ser_store (D2H)."""
        ser = clen.astype(np.uint64) + np.uint64(8)
        total = int(ser.sum())
        ptr, cap, at, tmp = self._ser_sink
        if at + total > cap:
            raise RuntimeError(f"ser_store too small: {at + total} > {cap} bytes")
        if tmp is None or tmp.numel() < total:
            tmp = ops.padded_empty(max(total, 1 << 30), arena.device)
            self._ser_sink[3] = tmp
        idx = np.arange(len(clen), dtype=np.uint64)
        addr = np.where(scheme > 0, np.uint64(frames.data_ptr()) + idx * np.uint64(ops.LZ4_SLOT),
                        np.uint64(arena.data_ptr()) + offs.astype(np.uint64))
        ops.pack_frames(addr, clen, lens, scheme, (np.cumsum(ser) - ser).astype(np.uint64), tmp)
        ops.hip().memcpy_async(ptr + at, tmp.data_ptr(), total, torch.cuda.current_stream(arena.device).cuda_stream)
        torch.cuda.synchronize(arena.device)  # tmp and frames are reused / freed next batch
        self._ser_sink[2] = at + total

    def pack_serialized(self, arena: torch.Tensor, a: int, b: int, out: torch.Tensor, out_off: np.ndarray) -> None:
        """Serialize chunks [a, b) ([8-byte header | stored payload], what the CAS serves) into `out`
        at out_off (GPU).  Compressed worlds compress the chunks again — the kernel is
        deterministic, so the frames are the ones the plan was sized with."""
        lens = self.chunk_len[a:b]
        if not self.chunk_scheme[a:b].any():
            ops.pack_chunks(arena, self.chunk_off[a:b], lens, out_off, out)
            return
        for s0 in range(a, b, 4096):  # bounded compression scratch (2 x LZ4_SLOT per chunk)
            s1 = min(b, s0 + 4096)
            frames, flen = ops.compress_chunks(arena, self.chunk_off[s0:s1], self.chunk_len[s0:s1], bg4=True)
            if not np.array_equal(np.where(flen > 0, flen, self.chunk_len[s0:s1]), self.chunk_clen[s0:s1]):
                raise RuntimeError("GPU compression is not reproducible")
            idx = np.arange(s1 - s0, dtype=np.uint64)
            addr = np.where(flen > 0, np.uint64(frames.data_ptr()) + idx * np.uint64(ops.LZ4_SLOT),
                            np.uint64(arena.data_ptr()) + self.chunk_off[s0:s1].astype(np.uint64))
            ops.pack_frames(addr, self.chunk_clen[s0:s1], self.chunk_len[s0:s1], self.chunk_scheme[s0:s1],
                            out_off[s0 - a:s1 - a], out)
            torch.cuda.synchronize(out.device)
            del frames

    # ------------------------------------------------------------------------------------------
    # Host build (tests / small models)
    # ------------------------------------------------------------------------------------------
    def build_on_host(self) -> dict[str, bytes]:
        if self.compression != "none":
            raise ValueError("compressed synthetic worlds are built on the GPU (build_on_device)")
        contents = {}
        offs, lens, fidx, hs = [], [], [], []
        for i, f in enumerate(self.xet_files):
            data = self.file_bytes_host(f)
            contents[f.path] = data
            ends = np.asarray(_core.chunk_ends(data), dtype=np.uint64)
            starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)
            offs.append(starts + np.uint64(f.arena_off))
            lens.append((ends - starts).astype(np.uint32))
            fidx.append(np.full(len(ends), i, dtype=np.int32))
            for a, b in zip(starts.tolist(), ends.tolist()):
                hs.append(np.frombuffer(_core.chunk_hash(data[a:b]), dtype=np.uint8))
        self._set_chunks(np.concatenate(offs), np.concatenate(lens), np.concatenate(fidx))
        self.chunk_hashes = np.stack(hs) if hs else np.zeros((0, 32), np.uint8)
        fh = []
        for i in range(len(self.xet_files)):
            a, n = int(self.file_chunk0[i]), int(self.file_nchunks[i])
            leaves = [(self.chunk_hashes[j].tobytes(), int(self.chunk_len[j])) for j in range(a, a + n)]
            fh.append(np.frombuffer(_core.file_hash(leaves), dtype=np.uint8))
        self.file_hashes = np.stack(fh)
        self._plan_xorbs()
        return contents

    # ------------------------------------------------------------------------------------------
    def _set_chunks(self, offs, lens, fidx):
        self.chunk_off = offs
        self.chunk_len = lens
        self.chunk_file = fidx
        nf = len(self.xet_files)
        self.file_nchunks = np.bincount(fidx, minlength=nf).astype(np.int64)
        self.file_chunk0 = np.concatenate([[0], np.cumsum(self.file_nchunks)[:-1]]).astype(np.int64)

    def merkle_jobs(self):
        return [(int(a), int(n)) for a, n in zip(self.file_chunk0, self.file_nchunks)]

    def file_hash_hex(self, i: int) -> str:
        return _core.xet_hex(self.file_hashes[i].tobytes())

    def _plan_xorbs(self) -> None:
        if self.chunk_clen is None:
            self.chunk_clen = self.chunk_len.astype(np.uint32)
            self.chunk_scheme = np.zeros(self.n_chunks, dtype=np.uint8)
        ser = self.chunk_clen.astype(np.uint64) + np.uint64(8)  # 8-byte chunk header + stored payload
        self.xorb_of = np.asarray(_core.plan_xorbs(ser, self.max_xorb_bytes, MAX_XORB_CHUNKS), dtype=np.int64)
        # offset of each chunk header inside its xorb
        cum = np.cumsum(ser) - ser
        first = np.concatenate([[True], self.xorb_of[1:] != self.xorb_of[:-1]])
        xorb_start = np.maximum.accumulate(np.where(first, cum, 0).astype(np.uint64))
        self.ser_off = (cum - xorb_start).astype(np.uint64)
        self.ser_len = ser
        self.n_xorbs = int(self.xorb_of[-1]) + 1 if len(self.xorb_of) else 0
        self.xorb_chunk0 = np.flatnonzero(first).astype(np.int64)
        # terms: maximal runs of consecutive chunks sharing (file, xorb)
        brk = np.concatenate([[True], (self.xorb_of[1:] != self.xorb_of[:-1]) |
                              (self.chunk_file[1:] != self.chunk_file[:-1])])
        t0 = np.flatnonzero(brk)
        t1 = np.concatenate([t0[1:], [self.n_chunks]])
        T = np.zeros(len(t0), dtype=[("file", "<i4"), ("xorb", "<i8"), ("c0", "<i8"), ("c1", "<i8"),
                                     ("local0", "<i8"), ("ser0", "<u8"), ("ser_len", "<u8"),
                                     ("dst", "<u8"), ("ulen", "<u8")])
        T["file"] = self.chunk_file[t0]
        T["xorb"] = self.xorb_of[t0]
        T["c0"] = t0
        T["c1"] = t1
        T["local0"] = t0 - self.xorb_chunk0[self.xorb_of[t0]]
        T["ser0"] = self.ser_off[t0]
        cs = np.concatenate([[0], np.cumsum(ser)]).astype(np.uint64)
        T["ser_len"] = cs[t1] - cs[t0]
        T["dst"] = self.chunk_off[t0]
        cl = np.concatenate([[0], np.cumsum(self.chunk_len.astype(np.uint64))]).astype(np.uint64)
        T["ulen"] = cl[t1] - cl[t0]
        self.terms = T

    # ------------------------------------------------------------------------------------------
    def reconstruction(self, file_idx: int, cas_url: str) -> dict:
        """Xet reconstruction JSON for one file (CAS /v1/reconstructions/{file_hash})."""
        T = self.terms[self.terms["file"] == file_idx]
        terms, fetch = [], {}
        for t in T:
            xh = self.xorb_hash_hex(int(t["xorb"]))
            n = int(t["c1"] - t["c0"])
            local0 = int(t["local0"])
            terms.append({"hash": xh, "unpacked_length": int(t["ulen"]),
                          "range": {"start": local0, "end": local0 + n}})
            fetch.setdefault(xh, []).append({
                "range": {"start": local0, "end": local0 + n},
                "url": f"{cas_url}/xorbs/default/{xh}",
                "url_range": {"start": int(t["ser0"]), "end": int(t["ser0"] + t["ser_len"]) - 1}})
        return {"offset_into_first_range": 0, "terms": terms, "fetch_info": fetch}

    def xorb_hash(self, x: int) -> bytes:
        a = int(self.xorb_chunk0[x])
        b = int(self.xorb_chunk0[x + 1]) if x + 1 < self.n_xorbs else self.n_chunks
        leaves = [(self.chunk_hashes[j].tobytes(), int(self.chunk_len[j])) for j in range(a, b)]
        return _core.merkle_root(leaves)

    def xorb_hash_hex(self, x: int) -> str:
        if not hasattr(self, "_xorb_hex"):
            self._xorb_hex = {}
        if x not in self._xorb_hex:
            self._xorb_hex[x] = _core.xet_hex(self.xorb_hash(x))
        return self._xorb_hex[x]

    def xorb_bytes_host(self, x: int, contents: dict[str, bytes], policy: str = "none", footer: bool = True) -> bytes:
        """Serialize xorb x from host file contents (CAS object bytes)."""
        a = int(self.xorb_chunk0[x])
        b = int(self.xorb_chunk0[x + 1]) if x + 1 < self.n_xorbs else self.n_chunks
        bld = _core.XorbBuilder(policy)
        for j in range(a, b):
            f = self.xet_files[int(self.chunk_file[j])]
            rel = int(self.chunk_off[j]) - f.arena_off
            bld.add_chunk(contents[f.path][rel:rel + int(self.chunk_len[j])])
        return bld.serialize(footer)


def _host_fill(out: np.ndarray, seed: int, mode: int) -> None:
    """numpy twin of the device generator (zest_amd.ops.fill_synthetic) for small files."""
    n = out.size
    if n == 0:
        return
    M = np.uint64(0xFFFFFFFFFFFFFFFF)

    def splitmix(x):
        x = (x + np.uint64(0x9E3779B97F4A7C15)) & M
        x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M
        x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M
        return x ^ (x >> np.uint64(31))

    with np.errstate(over="ignore"):
        if mode == 0:
            words = (n + 7) // 8
            idx = np.arange(words, dtype=np.uint64)
            w = splitmix(np.uint64(seed) ^ (idx * np.uint64(0xD1B54A32D192ED03)))
            out[:] = w.view(np.uint8)[:n]
        else:
            ne = (n + 1) // 2
            e = np.arange(ne, dtype=np.uint64)
            h = splitmix(np.uint64(seed) ^ (e * np.uint64(0xA24BAED4963EE407)))
            u1 = (((h >> np.uint64(40)) & np.uint64(0xFFFFFF)).astype(np.float32) + 0.5) / 16777216.0
            u2 = ((h >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.float32) / 16777216.0
            z = (np.sqrt(-2.0 * np.log(u1)) * np.cos(6.28318530718 * u2) * 0.02).astype(np.float32)
            bits = z.view(np.uint32)
            bf = ((bits + np.uint32(0x7FFF) + ((bits >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16)).astype(np.uint16)
            out[:] = bf.view(np.uint8)[:n]
