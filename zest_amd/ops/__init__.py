"""Torch-facing wrappers of the HIP/CDNA4 kernels (zest_amd._hip) with CPU oracles.

Every op validates shapes, dtypes, devices and buffer padding on the host BEFORE launching, so a
bad descriptor can never become an out-of-bounds GPU access.  GPU tensors always take the HIP path
(there is no silent eager fallback: if the extension is missing on a GPU box the import raises);
CPU tensors take the C++ host oracle in zest_amd._core, which is what the gloo/CPU tests use.

Kernel map: K1 hash_ranges/hash_placed, K2 merkle_roots, K3+K4 ingest_terms,
K5 cdc_candidates, K7 pack_chunks.
"""
from __future__ import annotations

import functools
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import _core

PAD = 4096  # bytes every device buffer must have past its logical end (kernels read whole lines)

TERM_DTYPE = np.dtype([("src", "<u8"), ("src_len", "<u8"), ("dst", "<u8"), ("chunk_base", "<u4"),
                       ("n_chunks", "<u4"), ("ulen", "<u8")])
CHUNK_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("clen", "<u4"), ("ulen", "<u4"),
                        ("scheme", "<u4"), ("term", "<u4")])
MERKLE_JOB_DTYPE = np.dtype([("leaf_base", "<u8"), ("n_leaves", "<u8"), ("want_file_hash", "<u4"),
                             ("pad", "<u4")])

ERR_NAMES = {0: "ok", 1: "bad chunk header", 2: "chunk out of range", 3: "chunk count/size mismatch",
             4: "malformed LZ4", 5: "decoded size mismatch", 6: "hash mismatch", 7: "chunk exceeds capacity"}


class IngestError(RuntimeError):
    def __init__(self, code: int, index: int):
        super().__init__(f"{ERR_NAMES.get(code, code)} at index {index}")
        self.code = code
        self.index = index


@functools.lru_cache(maxsize=1)
def hip():
    """The compiled HIP extension.  Raises (loudly) when it is missing or built for no GPU."""
    from .. import _hip  # noqa: F401  (ImportError propagates: no silent fallback)

    assert _hip.TERM_BYTES == TERM_DTYPE.itemsize, "ZgTerm layout drift"
    assert _hip.CHUNK_BYTES == CHUNK_DTYPE.itemsize, "ZgChunk layout drift"
    assert _hip.MERKLE_JOB_BYTES == MERKLE_JOB_DTYPE.itemsize, "ZgMerkleJob layout drift"
    return _hip


def mem_origin_add(hexes, starts, ptrs, lens) -> int:
    """Serve fetch_info URLs mem://<name>/<xorb hex> from host memory (csrc/core/hub.h): run i is
    bytes [starts[i], starts[i] + lens[i]) of xorb hexes[i], at address ptrs[i] (kept alive by the
    caller).  Registered in both native modules (each links its own host core): _core's host fetches
    and _hip's DeviceXetPull read the same origin."""
    args = (list(hexes), [int(x) for x in starts], [int(x) for x in ptrs], [int(x) for x in lens])
    n = _core.mem_origin_add(*args)
    try:
        from .. import _hip
    except ImportError:
        return n
    _hip.mem_origin_add(*args)
    return n


def mem_origin_clear() -> None:
    _core.mem_origin_clear()
    try:
        from .. import _hip
    except ImportError:
        return
    _hip.mem_origin_clear()


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def padded_empty(nbytes: int, device, pad: int = PAD) -> torch.Tensor:
    """uint8 buffer of `nbytes` logical bytes backed by nbytes + pad of storage."""
    base = torch.empty(nbytes + pad, dtype=torch.uint8, device=device)
    return base[:nbytes]


def vmm_empty(nbytes: int, device, pad: int = PAD, chunk: int = 512 << 20) -> torch.Tensor:
    """Like :func:`padded_empty`, but the storage is a HIP virtual-memory arena built from
    ``chunk``-sized physical allocations that other processes can map (engine.map_peer_arenas
    passes the chunks as dmabuf fds).  Imports of torch allocations of >= 2 GiB through
    hipIpcOpenMemHandle hung on the MI355X box; this path mapped 16 GiB in tens of ms
    (csrc/bind/hip_vmm.cpp)."""
    from torch.utils.dlpack import from_dlpack
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError("vmm_empty is for GPU arenas")
    m = hip().vmm_alloc(nbytes + pad, device.index if device.index is not None else torch.cuda.current_device(),
                        chunk)
    t = from_dlpack(m.dlpack(nbytes + pad))[:nbytes]
    t._zest_vmm = m  # the DLPack deleter keeps the mapping alive for every view; this finds it
    return t


def vmm_mapping(t: torch.Tensor):
    """The VmmMapping behind a tensor returned by :func:`vmm_empty` (None otherwise)."""
    return getattr(t, "_zest_vmm", None)


def _has_pad(t: torch.Tensor, pad: int = PAD) -> bool:
    st = t.untyped_storage().nbytes()
    end = (t.storage_offset() + t.numel()) * t.element_size()
    return st - end >= pad


def _as_padded_u8(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.uint8:
        t = t.view(torch.uint8) if t.is_contiguous() else t.contiguous().view(torch.uint8)
    t = t.reshape(-1)
    if not t.is_contiguous() or not _has_pad(t):
        p = padded_empty(t.numel(), t.device)
        p.copy_(t)
        t = p
    return t


def _dev_array(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(device, non_blocking=False)


# ----------------------------------------------------------------------------------------------
# K1: keyed BLAKE3 over (offset, len) ranges
# ----------------------------------------------------------------------------------------------
KEY_DATA, KEY_NODE, KEY_PLAIN, KEY_ZERO = 0, 1, 2, 3


def hash_ranges(buf: torch.Tensor, offsets, lens, key_mode: int = KEY_DATA) -> torch.Tensor:
    """Hash buf[off:off+len] for each range; returns uint8 [n, 32] on buf's device.

    key_mode: 0 Xet chunk (DATA_KEY), 1 Merkle node key, 2 plain BLAKE3, 3 all-zero key."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint32)
    n = len(offsets)
    if n == 0:
        return torch.empty((0, 32), dtype=torch.uint8, device=buf.device)
    if np.any(offsets + lens > buf.numel() * buf.element_size()):
        raise ValueError("hash range past end of buffer")
    if buf.device.type != "cuda":
        data = buf.reshape(-1).view(torch.uint8).numpy()
        keys = {KEY_DATA: _core.DATA_KEY, KEY_NODE: _core.INTERNAL_NODE_KEY, KEY_ZERO: bytes(32)}
        out = np.empty((n, 32), dtype=np.uint8)
        for i, (o, l) in enumerate(zip(offsets.tolist(), lens.tolist())):
            mv = data[o:o + l]
            h = _core.blake3(mv) if key_mode == KEY_PLAIN else _core.blake3_keyed(keys[key_mode], mv)
            out[i] = np.frombuffer(h, dtype=np.uint8)
        return torch.from_numpy(out)
    if np.any(lens > 128 * 1024):
        raise ValueError("device hash_ranges supports messages up to 128 KiB")
    H = hip()
    buf = _as_padded_u8(buf)
    offs_d = torch.from_numpy(offsets.view(np.int64).copy()).to(buf.device)
    lens_d = torch.from_numpy(lens.view(np.int32).copy()).to(buf.device)
    out = torch.empty((n, 32), dtype=torch.uint8, device=buf.device)
    sb = H.hash_scratch_bytes(n, int(lens.sum(dtype=np.uint64)))
    scratch = torch.empty(sb, dtype=torch.uint8, device=buf.device)
    H.hash_ranges(buf.data_ptr(), offs_d.data_ptr(), lens_d.data_ptr(), n, out.data_ptr(), key_mode,
                  _stream(buf.device), scratch.data_ptr(), sb)
    return out


class HashScratch:
    """Device scratch of the leaf-flat K1 pipeline (blake3_flat.hip), grown on demand.  Use one per
    stream, and call get() with that stream current: launches on one stream are ordered, so they
    can share the buffer, and when it grows the caching allocator hands the old block only to later
    allocations on that same stream, i.e. after the launches already queued on it."""

    def __init__(self, device, ingest: bool = False):
        self.device = torch.device(device)
        self.buf = None
        self.ingest = ingest  # an ingest launch's scratch (also the decoder's BG4 staging)

    def get(self, n: int, total_bytes: int) -> tuple[int, int]:
        H = hip()
        need = (H.ingest_scratch_bytes if self.ingest else H.hash_scratch_bytes)(int(n), int(total_bytes))
        if self.buf is None or self.buf.numel() < need:
            self.buf = torch.empty(need + (need >> 3), dtype=torch.uint8, device=self.device)
        return self.buf.data_ptr(), self.buf.numel()


class DecodeScratch:
    """Device scratch of the experimental two-kernel LZ4/BG4 decoder (lz4seq.hip k_lz4_parse +
    k_lz4_exec: per-chunk sequence records, 3 bytes per compressed byte), grown on demand; one per
    stream.  Only `hip().lz4_decode(..., rec_scratch=...)` uses it (kbench, tests): the ingest path
    runs the one-kernel batched decoder, which is faster end to end (profiles/lz4_records_r3.md)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf = None

    def get(self, n: int, src_bytes: int) -> tuple[int, int]:
        need = hip().lz4_rec_scratch_bytes(int(n), int(src_bytes))
        if self.buf is None or self.buf.numel() < need:
            self.buf = torch.empty(need + (need >> 3), dtype=torch.uint8, device=self.device)
        return self.buf.data_ptr(), self.buf.numel()


# ----------------------------------------------------------------------------------------------
# K3 + K4: ingest fetched xorb runs into a destination arena, then K1 chunk hashes
# ----------------------------------------------------------------------------------------------
@dataclass
class IngestPlan:
    """Host-side description of a batch of fetched runs, pre-validated against the buffers."""
    terms: np.ndarray  # TERM_DTYPE
    n_chunks: int

    @staticmethod
    def make(terms: np.ndarray) -> "IngestPlan":
        terms = np.ascontiguousarray(terms, dtype=TERM_DTYPE)
        n = int(terms["n_chunks"].sum()) if len(terms) else 0
        if len(terms) and np.any(terms["chunk_base"][1:] < terms["chunk_base"][:-1] + terms["n_chunks"][:-1]):
            raise ValueError("term chunk ranges overlap")
        return IngestPlan(terms, n)


class IngestWorkspace:
    """Reusable device descriptors/error word for repeated ingests on one device (no per-call
    allocation inside the timed loop)."""

    def __init__(self, device, max_terms: int, max_chunks: int):
        self.device = torch.device(device)
        self.max_terms = max_terms
        self.max_chunks = max_chunks
        self.terms = torch.empty(max_terms * TERM_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        self.chunks = torch.empty(max_chunks * CHUNK_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.terms_host = torch.empty(max_terms * TERM_DTYPE.itemsize, dtype=torch.uint8).pin_memory() \
            if self.device.type == "cuda" else None
        self._clip_scratch = None
        self.hash_scratch = HashScratch(self.device, ingest=True) if self.device.type == "cuda" else None

    def index_scratch(self, H, n_terms: int) -> tuple[int, int]:
        """(ptr, bytes) of this workspace's parallel header-walk scratch, grown to n_terms."""
        need = H.index_scratch_bytes(max(1, n_terms))
        if getattr(self, "_index_scratch", None) is None or self._index_scratch.numel() < need:
            self._index_scratch = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._index_scratch.data_ptr(), self._index_scratch.numel()

    def clip_scratch(self) -> int:
        """Device scratch for clipped decodes, private to this workspace (so to its stream)."""
        if self._clip_scratch is None:
            self._clip_scratch = torch.empty(hip().CLIP_SCRATCH_BYTES, dtype=torch.uint8, device=self.device)
        return self._clip_scratch.data_ptr()


FUSED_INGEST = os.environ.get("ZEST_FUSED_INGEST", "1") != "0"


# The parallel header walk is the default (ZEST_INDEX_SCAN=0: the serial walk).  History: it was
# opt-in after it measured slower than the serial walk (gpubench 256 MiB lz4_decode_gpu 3.96 -> 9.69
# ms, profiles/r5/gpubench256_scan_r5c.json): LZ4 streams of BG4 bf16 weights are full of header-like
# byte patterns.  Compressed candidates now need the LZ4 frame magic (millions of candidates -> a
# few), and the link picks the chain out of the candidates instead of handing any term with a
# look-alike to the serial walk (which every term of a 256 MiB batch had): scan 112 us + link 32 us
# against the serial walk's 761 us; lz4_decode_gpu 69.0 -> 85.4 GB/s, xorb_verify_gpu 267 -> 575
# GiB/s; the 70B engine bench is unchanged (64.34 / 64.30 GB/s serial / parallel: the walk is hidden
# under each round's H2D copy either way) (profiles/r5/index_scan_r5ab/).
INDEX_SCAN = os.environ.get("ZEST_INDEX_SCAN", "1") == "1"


def index_terms(H, src_ptr: int, src_n: int, terms_ptr: int, n_terms: int, chunks_ptr: int, err_ptr: int, stream: int,
                ws: "IngestWorkspace | None" = None) -> None:
    """Device header walk of n_terms runs in src[0, src_n) into chunk records (K4).  With a workspace
    for its scratch (and ZEST_INDEX_SCAN not 0): the parallel walk -- candidate-header scan of the
    span, per-term LDS sort/link + prefix sums (csrc/gpu/ingest.hip k_hdr_scan / k_hdr_link), serial
    fallback per term; identical records.  Otherwise one thread per term chases its headers (~0.5 ms
    per 64 MiB run whatever the GPU's width)."""
    if ws is not None and INDEX_SCAN and ws.device.type == "cuda":
        sp, sb = ws.index_scratch(H, n_terms)
        H.index_terms_scan(src_ptr, src_n, terms_ptr, n_terms, chunks_ptr, err_ptr, sp, sb, stream)
        return
    H.index_terms(src_ptr, terms_ptr, n_terms, chunks_ptr, err_ptr, stream)


def ingest_terms(src: torch.Tensor, dst: torch.Tensor, terms: np.ndarray, hashes: torch.Tensor,
                 hash_base: int = 0, clip=None, ws: IngestWorkspace | None = None,
                 check: bool = True, fused: bool | None = None, has_compressed: bool = True) -> None:
    """Decode + place + hash a batch of fetched runs.

    src: uint8 staging buffer holding the runs (padded); dst: uint8 arena (padded).
    terms: TERM_DTYPE records; chunk_base indexes `hashes` (uint8 [N, 32]) relative to hash_base.
    clip: optional (lo, hi) arena byte window this rank owns: bytes outside are not written, and
    the hashes of chunks not entirely inside the window are unspecified.
    LZ4 chunks take the batched decoder (lz4seq.hip) unless clipped (LDS-ring decoder).
    fused (default: ZEST_FUSED_INGEST != 0): unclipped batches run decode + one fused place/hash
    pass (zg_ingest_chunks) instead of place then hash; `has_compressed=False` skips the decoder.
    """
    terms = np.ascontiguousarray(terms, dtype=TERM_DTYPE)
    nt = len(terms)
    if nt == 0:
        return
    n_chunks = int((terms["chunk_base"] + terms["n_chunks"]).max())
    src_n = src.numel() * src.element_size()
    dst_n = dst.numel() * dst.element_size()
    if np.any(terms["src"] + terms["src_len"] > src_n):
        raise ValueError("term run past end of src buffer")
    if np.any((terms["ulen"] > 0) & (terms["dst"] + terms["ulen"] > dst_n)):
        raise ValueError("term output past end of dst buffer")
    if np.any(terms["ulen"] == 0):
        raise ValueError("terms must carry their expected uncompressed length")
    if hashes.shape[0] < hash_base + n_chunks or hashes.shape[1] != 32 or hashes.dtype != torch.uint8:
        raise ValueError("hashes buffer too small")
    lo, hi = (0, dst_n) if clip is None else (int(clip[0]), int(clip[1]))
    if src.device.type != "cuda":
        return _ingest_cpu(src, dst, terms, hashes, hash_base, lo, hi)
    H = hip()
    dev = src.device
    if dst.device != dev or hashes.device != dev:
        raise ValueError("src/dst/hashes must share a device")
    src = _as_padded_u8(src)
    if not _has_pad(dst.view(torch.uint8).reshape(-1)):
        raise ValueError("dst arena must be allocated with ops.padded_empty (needs PAD slack)")
    dst8 = dst.view(torch.uint8).reshape(-1)
    if ws is None or ws.max_terms < nt or ws.max_chunks < n_chunks:
        ws = IngestWorkspace(dev, nt, n_chunks)
    st = _stream(dev)
    tbytes = torch.from_numpy(terms.view(np.uint8).copy())
    if ws.terms_host is not None:
        ws.terms_host[: tbytes.numel()].copy_(tbytes)
        ws.terms[: tbytes.numel()].copy_(ws.terms_host[: tbytes.numel()], non_blocking=True)
    else:
        ws.terms[: tbytes.numel()].copy_(tbytes)
    ws.err.zero_()
    ws.chunks[: n_chunks * CHUNK_DTYPE.itemsize].zero_()  # gaps between terms become no-op descriptors
    index_terms(H, src.data_ptr(), src_n, ws.terms.data_ptr(), nt, ws.chunks.data_ptr(), ws.err.data_ptr(), st, ws)
    clipped = lo > 0 or hi < dst_n
    hptr = hashes.data_ptr() + 32 * hash_base
    sp, sb = ws.hash_scratch.get(n_chunks, int(terms["ulen"].sum()))
    if (FUSED_INGEST if fused is None else fused) and not clipped:
        H.ingest_chunks(src.data_ptr(), src_n, dst8.data_ptr(), dst_n, ws.chunks.data_ptr(), n_chunks,
                        has_compressed, ws.err.data_ptr(), hptr, 0, 0, st, sp, sb)
    else:
        H.place_chunks(src.data_ptr(), src_n, dst8.data_ptr(), dst_n, ws.chunks.data_ptr(), n_chunks, lo, hi,
                       ws.err.data_ptr(), st, ws.clip_scratch() if clipped else 0)
        H.hash_chunks(dst8.data_ptr(), dst_n, ws.chunks.data_ptr(), n_chunks, hptr, 0, 0, st, sp, sb)
    if check:
        raise_on_error(ws.err)


def raise_on_error(err: torch.Tensor) -> None:
    v = int(err.item())
    if v:
        raise IngestError(v >> 32, v & 0xFFFFFFFF)


def _ingest_cpu(src, dst, terms, hashes, hash_base, lo, hi):
    s = src.reshape(-1).view(torch.uint8).numpy()
    d = dst.reshape(-1).view(torch.uint8).numpy()
    for t in terms:
        run = s[int(t["src"]): int(t["src"] + t["src_len"])]
        idx = _core.index_chunks(run)
        if len(idx) != int(t["n_chunks"]):
            raise IngestError(3, 0)
        data, hs = _core.extract_chunk_range(run, 0, len(idx), True)
        if len(data) != int(t["ulen"]):
            raise IngestError(3, 0)
        a = int(t["dst"])
        b = a + len(data)
        wa, wb = max(a, lo), min(b, hi)
        if wa < wb:
            d[wa:wb] = np.frombuffer(data, dtype=np.uint8)[wa - a: wb - a]
        base = hash_base + int(t["chunk_base"])
        for i, (h, _) in enumerate(hs):
            hashes[base + i] = torch.from_numpy(np.frombuffer(h, dtype=np.uint8).copy())


def hash_placed(dst: torch.Tensor, chunk_offsets, chunk_lens) -> torch.Tensor:
    """Re-hash chunks already resident in an arena (verify-on-receive)."""
    return hash_ranges(dst, chunk_offsets, chunk_lens, KEY_DATA)


# ----------------------------------------------------------------------------------------------
# K2: Merkle roots / file hashes
# ----------------------------------------------------------------------------------------------
def merkle_roots(hashes: torch.Tensor, sizes: torch.Tensor, jobs, file_hash: bool = True) -> torch.Tensor:
    """jobs: list of (leaf_base, n_leaves). Returns uint8 [n_jobs, 32] roots (file hashes if
    `file_hash`).  hashes: uint8 [N, 32]; sizes: int64 [N]."""
    jobs = list(jobs)
    nj = len(jobs)
    if nj == 0:
        return torch.empty((0, 32), dtype=torch.uint8, device=hashes.device)
    N = hashes.shape[0]
    for b, n in jobs:
        if b < 0 or n < 0 or b + n > N:
            raise ValueError("merkle job out of range")
    if hashes.device.type != "cuda":
        hs = hashes.numpy()
        sz = sizes.numpy()
        out = np.empty((nj, 32), dtype=np.uint8)
        for j, (b, n) in enumerate(jobs):
            leaves = [(hs[i].tobytes(), int(sz[i])) for i in range(b, b + n)]
            r = _core.file_hash(leaves) if file_hash else _core.merkle_root(leaves)
            out[j] = np.frombuffer(r, dtype=np.uint8)
        return torch.from_numpy(out)
    H = hip()
    dev = hashes.device
    rec = np.zeros(nj, dtype=MERKLE_JOB_DTYPE)
    rec["leaf_base"] = [b for b, _ in jobs]
    rec["n_leaves"] = [n for _, n in jobs]
    rec["want_file_hash"] = 1 if file_hash else 0
    jobs_d = _dev_array(rec, dev)
    maxn = max(n for _, n in jobs)
    sb = H.merkle_scratch_bytes(maxn, nj)
    scratch = torch.empty(sb, dtype=torch.uint8, device=dev)
    roots = torch.empty((nj, 32), dtype=torch.uint8, device=dev)
    hashes = hashes.contiguous()
    sizes = sizes.to(torch.int64).contiguous()
    H.merkle(hashes.data_ptr(), sizes.data_ptr(), jobs_d.data_ptr(), nj, roots.data_ptr(), scratch.data_ptr(), sb,
             _stream(dev))
    return roots


# ----------------------------------------------------------------------------------------------
# K5 CDC, K7 pack, synthetic content
# ----------------------------------------------------------------------------------------------
XET_MASK = 0xFFFF << 48


def cdc_candidates(data: torch.Tensor, mask: int = XET_MASK, capacity: int | None = None) -> np.ndarray:
    """Sorted END offsets (i+1) whose 64-byte-window gear hash has (h & mask) == 0."""
    n = data.numel() * data.element_size()
    if data.device.type != "cuda":
        d = data.reshape(-1).view(torch.uint8).numpy().tobytes()
        out = []
        h = 0
        table = _gear_table()
        for i, b in enumerate(d):
            h = ((h << 1) + table[b]) & 0xFFFFFFFFFFFFFFFF
            if h & mask == 0:
                out.append(i + 1)
        return np.asarray(out, dtype=np.uint64)
    H = hip()
    data = _as_padded_u8(data)
    cap = capacity or max(1024, n // 4096)
    out = torch.empty(cap, dtype=torch.int64, device=data.device)
    count = torch.zeros(1, dtype=torch.int64, device=data.device)
    H.cdc_candidates(data.data_ptr(), n, mask, out.data_ptr(), count.data_ptr(), cap, _stream(data.device))
    k = int(count.item())
    if k > cap:
        return cdc_candidates(data, mask, k + 1024)
    return np.sort(out[:k].cpu().numpy().astype(np.uint64))


@functools.lru_cache(maxsize=1)
def _gear_table():
    # Recover the table from the host core (one value per byte via gear_window_hash of 1 byte).
    return [_core.gear_window_hash(bytes([b]), 0) for b in range(256)]


def select_chunks(candidates: np.ndarray, n: int, min_size: int = 8192, max_size: int = 131072) -> np.ndarray:
    """Apply the Xet min/max rule to sorted candidate END offsets -> chunk END offsets."""
    return np.asarray(_core.select_boundaries(np.ascontiguousarray(candidates, dtype=np.uint64), n, min_size,
                                              max_size), dtype=np.uint64)


def fill_synthetic(t: torch.Tensor, seed: int, stream_offset: int = 0, mode: int = 0) -> None:
    """Deterministic synthetic bytes: mode 0 uniform random, mode 1 bf16 ~ N(0, 0.02)."""
    H = hip()
    u8 = t.view(torch.uint8).reshape(-1)
    H.fill_synthetic(u8.data_ptr(), u8.numel(), seed & 0xFFFFFFFFFFFFFFFF, stream_offset, mode, _stream(t.device))


def sha1_info_hash(xorb_hashes: torch.Tensor) -> torch.Tensor:
    """uint8 [n, 32] xorb hashes -> uint8 [n, 20] BitTorrent info-hashes (K6)."""
    n = xorb_hashes.shape[0]
    if xorb_hashes.device.type != "cuda":
        hs = xorb_hashes.numpy()
        return torch.from_numpy(np.stack([np.frombuffer(_core.info_hash(hs[i].tobytes()), dtype=np.uint8)
                                          for i in range(n)]) if n else np.zeros((0, 20), np.uint8))
    src = xorb_hashes.contiguous()
    out = torch.empty((n, 20), dtype=torch.uint8, device=src.device)
    hip().sha1_info_hash(src.data_ptr(), n, out.data_ptr(), _stream(src.device))
    return out


def pack_chunks(data: torch.Tensor, data_off: np.ndarray, lens: np.ndarray, out_off: np.ndarray,
                out: torch.Tensor) -> None:
    """Serialize uncompressed chunks (8-byte header + payload) into `out` at out_off."""
    n = len(lens)
    if n == 0:
        return
    data_n = data.numel()
    out_n = out.numel()
    data_off = np.asarray(data_off, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint32)
    out_off = np.asarray(out_off, dtype=np.uint64)
    if np.any(data_off + lens > data_n) or np.any(out_off + lens + 8 > out_n):
        raise ValueError("pack_chunks range out of bounds")
    if np.any(lens >= (1 << 24)):
        raise ValueError("chunk too large for a u24 header")
    H = hip()
    dev = data.device
    data = _as_padded_u8(data)
    d_off = torch.from_numpy(data_off.view(np.int64).copy()).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32).copy()).to(dev)
    o_off = torch.from_numpy(out_off.view(np.int64).copy()).to(dev)
    H.pack_chunks(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), o_off.data_ptr(), n, out.data_ptr(),
                  _stream(dev))


# ----------------------------------------------------------------------------------------------
# K7b: chunk compression (BG4 grouping + LZ4 frame) and serialization of compressed chunks
# ----------------------------------------------------------------------------------------------
LZ4_SLOT = 132 << 10  # device bytes per chunk for one frame (>= LZ4 bound of 128 KiB + frame overhead)


@functools.lru_cache(maxsize=1)
def _lz4_header_checksums() -> tuple[int, int]:
    """Frame-descriptor checksum bytes the host encoder writes for 64 KiB / 256 KiB blocks."""
    return _core.lz4_compress_frame(b"\0" * 16)[6], _core.lz4_compress_frame(b"\0" * 65537)[6]


def compress_chunks(buf: torch.Tensor, offsets, lens, bg4: bool = True):
    """Compress each chunk buf[off:off+len] on the GPU into an LZ4 frame (BG4-grouped first when
    `bg4`), the layout the host encoder and hf_xet use.  Returns (frames, frame_len): frames is a
    device buffer holding chunk i's frame at i * LZ4_SLOT; frame_len[i] == 0 means the chunk does
    not compress and is stored raw (scheme 0), as Xet does."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint32)
    n = len(offsets)
    if buf.device.type != "cuda":
        raise ValueError("compress_chunks runs on the GPU")
    if n and (np.any(lens > 128 * 1024) or np.any(offsets + lens > buf.numel() * buf.element_size())):
        raise ValueError("compress_chunks: chunk larger than 128 KiB or past the buffer")
    dev = buf.device
    frames = padded_empty(max(1, n) * LZ4_SLOT, dev)
    flen = torch.zeros(max(1, n), dtype=torch.int32, device=dev)
    if n:
        H = hip()
        buf = _as_padded_u8(buf)
        scratch = padded_empty(n * LZ4_SLOT if bg4 else 1, dev)
        offs_d = torch.from_numpy(offsets.view(np.int64).copy()).to(dev)
        lens_d = torch.from_numpy(lens.view(np.int32).copy()).to(dev)
        hc64, hc256 = _lz4_header_checksums()
        H.compress_chunks(buf.data_ptr(), offs_d.data_ptr(), lens_d.data_ptr(), n, int(bg4), scratch.data_ptr(),
                          LZ4_SLOT, frames.data_ptr(), LZ4_SLOT, flen.data_ptr(), hc64, hc256,
                          torch.cuda.current_stream(dev).cuda_stream)
    return frames, flen[:n].cpu().numpy().astype(np.int64)


def pack_frames(src_addr: np.ndarray, clen: np.ndarray, ulen: np.ndarray, scheme: np.ndarray, out_off: np.ndarray,
                out: torch.Tensor) -> None:
    """Serialize chunks whose payload (compressed frame or raw bytes) sits at device address
    src_addr[i]: 8-byte header [0][clen u24][scheme][ulen u24] + payload, into `out` at out_off[i]."""
    n = len(clen)
    if n == 0:
        return
    clen = np.asarray(clen, dtype=np.uint32)
    out_off = np.asarray(out_off, dtype=np.uint64)
    if np.any(out_off + clen + 8 > out.numel()):
        raise ValueError("pack_frames range out of bounds")
    dev = out.device
    H = hip()
    t = [torch.from_numpy(np.ascontiguousarray(a).copy()).to(dev) for a in
         (np.asarray(src_addr, dtype=np.uint64).view(np.int64), clen.view(np.int32),
          np.asarray(ulen, dtype=np.uint32).view(np.int32), np.asarray(scheme, dtype=np.uint8),
          out_off.view(np.int64))]
    H.pack_frames(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), t[4].data_ptr(), n,
                  out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
