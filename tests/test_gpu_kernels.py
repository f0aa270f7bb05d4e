"""Numerics of the HIP/CDNA4 kernels vs the C++ host oracle (bit-exact: hashes and bytes).

Marked `gpu`: runs on a real MI355X.  The same ops also have CPU paths (tested in
test_ops_cpu.py) that the gloo multi-process tests use.
"""
import random

import numpy as np
import pytest
import torch

from zest_amd import _core as C
from zest_amd import ops

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.hip()  # must load: no silent fallback


def _bf16(n, seed=0):
    w = np.random.default_rng(seed).standard_normal(n).astype(np.float32) * 0.02
    return (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()


def test_hash_ranges_matches_cpu_all_sizes_and_alignments():
    rng = random.Random(1)
    data = rng.randbytes(1 << 21)
    buf = ops.padded_empty(len(data), DEV)
    buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    sizes = [0, 1, 3, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 4097, 8192, 65535, 65536, 65537, 100_000,
             131_071, 131_072]
    offs, lens = [], []
    for s in sizes:
        for a in range(4):
            offs.append(1000 + a + 7 * len(offs))
            lens.append(s)
    for _ in range(200):
        lens.append(rng.randint(0, 131_072))
        offs.append(rng.randint(0, len(data) - 131_072))
    got = ops.hash_ranges(buf, offs, lens).cpu().numpy()
    for i, (o, l) in enumerate(zip(offs, lens)):
        assert got[i].tobytes() == C.chunk_hash(data[o:o + l]), (o, l)
    # other key modes
    got_plain = ops.hash_ranges(buf, offs[:40], lens[:40], ops.KEY_PLAIN).cpu().numpy()
    got_node = ops.hash_ranges(buf, offs[:40], lens[:40], ops.KEY_NODE).cpu().numpy()
    for i in range(40):
        o, l = offs[i], lens[i]
        assert got_plain[i].tobytes() == C.blake3(data[o:o + l])
        assert got_node[i].tobytes() == C.internal_node_hash(data[o:o + l])


def _raw_hash_ranges(buf, offs, lens, key_mode=ops.KEY_DATA, scratch_bytes=None):
    """K1 straight through the binding: leaf-flat pipeline when scratch_bytes != 0, else the
    wave-per-message kernel."""
    H = ops.hip()
    n = len(offs)
    offs_d = torch.tensor(np.asarray(offs, dtype=np.int64), device=DEV)
    lens_d = torch.tensor(np.asarray(lens, dtype=np.uint32).view(np.int32), device=DEV)
    out = torch.full((n, 32), 0x5A, dtype=torch.uint8, device=DEV)
    sb = H.hash_scratch_bytes(n, int(np.asarray(lens, dtype=np.uint64).sum())) if scratch_bytes is None else scratch_bytes
    scratch = torch.full((max(sb, 1),), 0xA5, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    H.hash_ranges(buf.data_ptr(), offs_d.data_ptr(), lens_d.data_ptr(), n, out.data_ptr(), key_mode, st,
                  scratch.data_ptr() if sb else 0, sb)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_hash_leaf_flat_vs_wave_kernel_cdc_sizes():
    """Both K1 paths bit-exact vs the host oracle on CDC-like sizes: 8-128 KiB with every tree depth,
    one-leaf and empty messages, odd alignments, n not a multiple of the 8-chunk tree group, runs
    of tiny messages that put up to 64 owners in one leaf task."""
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 24 << 20, dtype=np.uint8).tobytes()
    buf = ops.padded_empty(len(data), DEV)
    buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    lens = list(rng.integers(8 << 10, (128 << 10) + 1, 300)) + [131_072] * 9 + [1, 0, 1024, 1025, 2048, 3] \
        + [int(x) for x in rng.integers(0, 1025, 150)] + list(rng.integers(8 << 10, 64 << 10, 7))
    offs, pos = [], 3
    for ln in lens:
        offs.append(pos)
        pos += int(ln) + int(rng.integers(0, 5))
    assert pos < len(data)
    want = [C.chunk_hash(data[o:o + int(ln)]) for o, ln in zip(offs, lens)]
    flat = _raw_hash_ranges(buf, offs, lens)
    wave = _raw_hash_ranges(buf, offs, lens, scratch_bytes=0)
    for i in range(len(lens)):
        assert flat[i].tobytes() == want[i], ("flat", i, lens[i])
        assert wave[i].tobytes() == want[i], ("wave", i, lens[i])
    # plain / node keys through the flat path
    sub = slice(0, 24)
    plain = _raw_hash_ranges(buf, offs[sub], lens[sub], ops.KEY_PLAIN)
    node = _raw_hash_ranges(buf, offs[sub], lens[sub], ops.KEY_NODE)
    for i, (o, ln) in enumerate(zip(offs[sub], lens[sub])):
        assert plain[i].tobytes() == C.blake3(data[o:o + int(ln)])
        assert node[i].tobytes() == C.internal_node_hash(data[o:o + int(ln)])


def test_hash_leaf_flat_multi_tile_plan():
    """The leaf plan runs as per-tile sums + per-tile scans over many workgroups (1024 chunks per
    tile): a launch of 3333 messages spans 4 tiles, the last one partial, with tile sums that differ
    (tiny messages in one tile, 64-128 KiB ones in another)."""
    rng = np.random.default_rng(11)
    lens = ([int(x) for x in rng.integers(0, 2049, 1100)] + [int(x) for x in rng.integers(64 << 10, (128 << 10) + 1, 200)]
            + [int(x) for x in rng.integers(0, 9000, 2033)])
    total = sum(lens) + 2 * len(lens) + 64
    data = rng.integers(0, 256, total, dtype=np.uint8).tobytes()
    buf = ops.padded_empty(len(data), DEV)
    buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    offs, pos = [], 1
    for ln in lens:
        offs.append(pos)
        pos += ln + int(rng.integers(0, 2))
    assert pos <= len(data)
    flat = _raw_hash_ranges(buf, offs, lens)
    for i, (o, ln) in enumerate(zip(offs, lens)):
        assert flat[i].tobytes() == C.chunk_hash(data[o:o + ln]), (i, ln)


def test_hash_leaf_flat_oversize_and_undersized_scratch():
    data = bytes(range(256)) * 4096
    buf = ops.padded_empty(len(data), DEV)
    buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    offs, lens = [0, 10, 20], [5000, 131_073, 70_000]
    got = _raw_hash_ranges(buf, offs, lens)
    assert got[0].tobytes() == C.chunk_hash(data[:5000])
    assert got[1].tobytes() == b"\xff" * 32  # over 128 KiB: rejected like the wave kernel does
    assert got[2].tobytes() == C.chunk_hash(data[20:70_020])
    # scratch sized for far fewer leaves than the launch has: every hash is all-ones (cannot verify)
    small = ops.hip().hash_scratch_bytes(3, 2048)
    bad = _raw_hash_ranges(buf, [0, 100, 200], [65_536, 65_536, 65_536], scratch_bytes=small)
    assert all(bad[i].tobytes() == b"\xff" * 32 for i in range(3))


def test_hash_chunks_flat_matches_wave_kernel_on_ingest():
    data, ends, b = _make_runs("none", 3)
    run = b.serialize(False)
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(run), 0, 0, len(ends), len(data))
    src = ops.padded_empty(len(run), DEV)
    src.copy_(torch.frombuffer(bytearray(run), dtype=torch.uint8))
    dst = ops.padded_empty(len(data), DEV)
    hashes = torch.zeros((len(ends), 32), dtype=torch.uint8, device=DEV)
    ws = ops.IngestWorkspace(DEV, 1, len(ends))
    ops.ingest_terms(src, dst, terms, hashes, ws=ws)  # flat path (workspace scratch)
    H = ops.hip()
    wave = torch.zeros_like(hashes)
    sizes = torch.zeros(len(ends), dtype=torch.int64, device=DEV)
    H.hash_chunks(dst.data_ptr(), dst.numel(), ws.chunks.data_ptr(), len(ends), wave.data_ptr(), sizes.data_ptr(), 0,
                  torch.cuda.current_stream().cuda_stream)
    assert torch.equal(hashes, wave)
    prev = 0
    want = []
    for e in ends:
        want.append(C.chunk_hash(data[prev:e]))
        prev = e
    assert [hashes[i].cpu().numpy().tobytes() for i in range(len(ends))] == want
    assert sizes.cpu().tolist() == list(np.diff([0] + list(ends)))


def _make_runs(policy, seed=0):
    rng = random.Random(seed)
    parts = [rng.randbytes(700_000), _bf16(400_000, seed), b"zest xorb ingest test line. " * 20_000,
             bytes(300_000)]
    data = b"".join(parts)
    ends = C.chunk_ends(data)
    b = C.XorbBuilder(policy)
    prev = 0
    for e in ends:
        b.add_chunk(data[prev:e])
        prev = e
    return data, ends, b


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("policy", ["none", "lz4", "bg4", "auto"])
def test_ingest_matches_cpu(policy, fused):
    """Ingest (decode + place + hash) vs the host builder, at odd src/dst offsets; `fused`: the one-
    pass place+hash (zg_ingest_chunks, raw chunks copied by the hashing waves) vs place then hash."""
    data, ends, b = _make_runs(policy)
    body = b.serialize(False)
    nck = len(ends)
    # Split the run into 3 terms at chunk boundaries; place them at odd src/dst offsets.
    bounds = b.chunk_boundaries()
    cuts = [0, nck // 3, 2 * nck // 3, nck]
    src_gap, dst_gap = 13, 7
    src = ops.padded_empty(len(body) + 64, DEV)
    terms = np.zeros(3, dtype=ops.TERM_DTYPE)
    src_host = bytearray(len(body) + 64)
    soff = src_gap
    uoffs = [0] + list(ends)
    for t in range(3):
        c0, c1 = cuts[t], cuts[t + 1]
        r0 = 0 if c0 == 0 else bounds[c0 - 1]
        r1 = bounds[c1 - 1]
        run = body[r0:r1]
        src_host[soff:soff + len(run)] = run
        terms[t] = (soff, len(run), dst_gap + uoffs[c0], c0, c1 - c0, uoffs[c1] - uoffs[c0])
        soff += len(run) + 3
    src = ops.padded_empty(len(src_host), DEV)
    src.copy_(torch.frombuffer(src_host, dtype=torch.uint8))
    dst = ops.padded_empty(len(data) + 2 * dst_gap, DEV)
    dst.fill_(0xAB)
    hashes = torch.zeros((nck, 32), dtype=torch.uint8, device=DEV)
    ops.ingest_terms(src, dst, terms, hashes, fused=fused, has_compressed=policy != "none")
    torch.cuda.synchronize()
    out = dst.cpu().numpy().tobytes()
    assert out[dst_gap:dst_gap + len(data)] == data
    assert out[:dst_gap] == b"\xab" * dst_gap and out[dst_gap + len(data):] == b"\xab" * dst_gap
    want = b"".join(b.chunk_hashes())
    assert hashes.cpu().numpy().tobytes() == want


@pytest.mark.parametrize("policy", ["bg4", "auto"])
def test_decoder_hash_matches_place_hash(policy, monkeypatch):
    """The LZ4 pair decoder hashing each chunk it decodes (default) vs the place/hash pass hashing
    every chunk (ZG_FUSED_HASH=0): same bytes, hashes and sizes, at a hash index base, for a batch
    of compressed and stored chunks; both equal the host builder's."""
    data, ends, b = _make_runs(policy, seed=5)
    body = b.serialize(False)
    nck = len(ends)
    rec = np.zeros(nck, dtype=ops.CHUNK_DTYPE)
    H = ops.hip()
    src = ops.padded_empty(len(body), DEV)
    src.copy_(torch.frombuffer(bytearray(body), dtype=torch.uint8))
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(body), 0, 0, nck, len(data))
    ws = ops.IngestWorkspace(DEV, 1, nck)
    terms_d = torch.from_numpy(terms.view(np.uint8).copy()).to(DEV)
    ops.index_terms(H, src.data_ptr(), len(body), terms_d.data_ptr(), 1, ws.chunks.data_ptr(), ws.err.data_ptr(),
                    torch.cuda.current_stream().cuda_stream, ws)
    torch.cuda.synchronize()
    rec[:] = np.frombuffer(ws.chunks[: nck * ops.CHUNK_DTYPE.itemsize].cpu().numpy().tobytes(), dtype=ops.CHUNK_DTYPE)
    assert (rec["scheme"] != 0).any()
    if policy == "auto":
        assert (rec["scheme"] == 0).any()
    base = 5
    got = {}
    # (fused hash, BG4 staging, chunk schedule): staged decode writes the grouped stream to the scratch
    # slice and the final bytes once (ingest scratch); unstaged scatters straight into place; the
    # dynamic schedule (work counter in the scratch) and the static one decode the same bytes, and so
    # does the parse without its L2 stream prefetch
    for env, stage, dyn, pf in (("1", "1", "1", "1"), ("1", "0", "1", "1"), ("0", "1", "1", "1"), ("1", "1", "0", "1"),
                                ("1", "1", "1", "0")):
        monkeypatch.setenv("ZG_FUSED_HASH", env)
        monkeypatch.setenv("ZG_BG4_STAGE", stage)
        monkeypatch.setenv("ZG_PAIR_DYNAMIC", dyn)
        monkeypatch.setenv("ZG_PAIR_PREFETCH", pf)
        dst = ops.padded_empty(len(data), DEV)
        dst.fill_(0x3C)
        hashes = torch.full((nck + base, 32), 0x77, dtype=torch.uint8, device=DEV)
        sizes = torch.full((nck + base,), -1, dtype=torch.int64, device=DEV)
        err = torch.zeros(1, dtype=torch.int64, device=DEV)
        sp, sb = ops.HashScratch(DEV, ingest=True).get(nck, len(data))
        H.ingest_chunks(src.data_ptr(), len(body), dst.data_ptr(), len(data), ws.chunks.data_ptr(), nck, True,
                        err.data_ptr(), hashes.data_ptr(), sizes.data_ptr(), base,
                        torch.cuda.current_stream().cuda_stream, sp, sb)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        assert dst.cpu().numpy().tobytes() == data, (env, stage, dyn, pf)
        got[env + stage + dyn + pf] = (hashes.cpu().numpy(), sizes.cpu().numpy())
    monkeypatch.delenv("ZG_FUSED_HASH")
    monkeypatch.delenv("ZG_BG4_STAGE")
    monkeypatch.delenv("ZG_PAIR_DYNAMIC")
    monkeypatch.delenv("ZG_PAIR_PREFETCH")
    (h1, s1), (h0, s0), (hu, su), (hs, ss) = got["1111"], got["0111"], got["1011"], got["1101"]
    hp, sp_ = got["1110"]
    assert np.array_equal(h1, h0) and np.array_equal(s1, s0)
    assert np.array_equal(h1, hu) and np.array_equal(s1, su)
    assert np.array_equal(h1, hs) and np.array_equal(s1, ss)
    assert np.array_equal(h1, hp) and np.array_equal(s1, sp_)
    assert h1[base:].tobytes() == b"".join(b.chunk_hashes())
    assert (h1[:base] == 0x77).all() and (s1[:base] == -1).all()
    assert s1[base:].tolist() == list(np.diff([0] + list(ends)))


def test_fused_ingest_places_exact_bytes():
    """The fused place+hash pass (zg_ingest_chunks, raw chunks copied by the hashing waves) at
    misaligned src/dst offsets: every in-bounds raw chunk lands byte-exact and hashes like the host
    oracle of its arena bytes; a descriptor past the arena is not placed, hashes as empty and is
    reported as ZG_ERR_RANGE at its index (the fused path used to drop it silently)."""
    rng = np.random.default_rng(31)
    sizes = [40_001, 65_536, 8_191, 131_072, 77_777, 1]
    data = [rng.bytes(n) for n in sizes]
    src_host = bytearray(3)
    rec = np.zeros(len(sizes), dtype=ops.CHUNK_DTYPE)
    dpos = 5
    for i, d in enumerate(data):
        src_host += b"\0" * 8  # the chunk header slot (payload follows it)
        rec[i] = (len(src_host), dpos, len(d), len(d), 0, 0)
        src_host += d + b"\x11" * (i % 3)
        dpos += len(d) + 7
    dst_n = dpos
    bad = 3
    rec[bad]["dst"] = dst_n - 3  # in the last gap, running past the arena end
    src = ops.padded_empty(len(src_host), DEV)
    src.copy_(torch.frombuffer(src_host, dtype=torch.uint8))
    dst = ops.padded_empty(dst_n, DEV)
    dst.fill_(0xCD)
    chunks = torch.from_numpy(rec.view(np.uint8).copy()).to(DEV)
    hashes = torch.zeros((len(sizes), 32), dtype=torch.uint8, device=DEV)
    err = torch.zeros(1, dtype=torch.int64, device=DEV)
    H = ops.hip()
    scr = ops.HashScratch(DEV)
    sp, sb = scr.get(len(sizes), sum(sizes))
    H.ingest_chunks(src.data_ptr(), src.numel(), dst.data_ptr(), dst_n, chunks.data_ptr(), len(sizes), False,
                    err.data_ptr(), hashes.data_ptr(), 0, 0, torch.cuda.current_stream().cuda_stream, sp, sb)
    torch.cuda.synchronize()
    assert int(err.item()) == (2 << 32) | bad, hex(int(err.item()))
    out = dst.cpu().numpy().tobytes()
    got = hashes.cpu().numpy()
    for i, d in enumerate(data):
        o = int(rec[i]["dst"])
        if i == bad:
            assert out[o:dst_n] == b"\xcd" * (dst_n - o)  # not placed
            # hashed over its planned leaves with no bytes: never the chunk's hash, so the file's
            # Merkle check fails too (the error word above is the primary report)
            assert got[i].tobytes() != C.chunk_hash(d)
            continue
        assert out[o:o + len(d)] == d, i
        assert got[i].tobytes() == C.chunk_hash(out[o:o + len(d)]), i


def _decode_both(body, chunks_data, n):
    """Index one run, then decode it with the one-kernel batched decoder and with the two-kernel
    records decoder; returns (output, error word) per decoder."""
    H = ops.hip()
    data = b"".join(chunks_data)
    src = ops.padded_empty(len(body) + 5, DEV)
    src.zero_()
    src[5:5 + len(body)].copy_(torch.frombuffer(bytearray(body), dtype=torch.uint8))
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (5, len(body), 3, 0, n, len(data))
    dst = ops.padded_empty(len(data) + 3, DEV)
    ws = ops.IngestWorkspace(DEV, 1, n)
    hashes = torch.zeros((n, 32), dtype=torch.uint8, device=DEV)
    ops.ingest_terms(src, dst, terms, hashes, ws=ws, check=False)  # leaves the chunk records in ws.chunks
    st = torch.cuda.current_stream().cuda_stream
    dec = ops.DecodeScratch(DEV)
    out = []
    for rec in (False, True, "pair"):
        dst.fill_(0x5A)
        ws.err.zero_()
        sp, sb = dec.get(n, src.numel()) if rec is True else (0, 0)
        H.lz4_decode(src.data_ptr(), src.numel(), dst.data_ptr(), dst.numel(), ws.chunks.data_ptr(), n,
                     ws.err.data_ptr(), st, 0, sp, sb, rec == "pair")
        torch.cuda.synchronize()
        out.append((dst.cpu().numpy().tobytes()[3:3 + len(data)], int(ws.err.item())))
    # the records decoder left per-chunk record counts at the head of its scratch (read below)
    # per-chunk record counts the parse left at the head of the scratch (-1: decode_chunk fallback)
    counts = dec.buf[:4 * n].view(torch.int32).cpu().tolist()
    return out, counts


@pytest.mark.parametrize("policy", ["lz4", "bg4"])
def test_lz4_records_decoder_matches_batched(policy):
    """Two-kernel decoder (lane-per-chunk parse into records + record-driven execute) vs the one-
    kernel batched decoder and the input: literal runs over the 14-bit record field, matches over
    0x7FFF (split records), tiny chunks whose record region is too small (decode_chunk fallback),
    BG4 groups of odd sizes; and a corrupted frame gives both decoders the same error word."""
    rng = np.random.default_rng(21)
    chunks = [b"a" * 40, b"xyz" * 9 + b"q", rng.bytes(40_000) + bytes(30_001), bytes(100_000),
              _bf16(32_771, 3)[:65_541], (b"zest " * 30_000)[:131_072], rng.bytes(20_000) * 3, bytes(1),
              b"ab" * 5000 + rng.bytes(17_000), rng.bytes(9_000)]
    b = C.XorbBuilder(policy)
    for ch in chunks:
        b.add_chunk(ch)
    body = b.serialize(False)
    idx = C.index_chunks(body)
    schemes = [e[2] for e in idx]
    assert sum(s != 0 for s in schemes) >= 6, schemes
    data = b"".join(chunks)
    ((ob, eb), (orc, er), (opr, epr)), counts = _decode_both(body, chunks, len(chunks))
    assert eb == 0 and er == 0 and epr == 0
    # the records path really ran: every compressed chunk of >= 256 stored bytes parsed into records
    for e, cnt in zip(idx, counts):
        if e[2] != 0 and e[1] >= 256:
            assert cnt > 0, (e, cnt)
    pos = 0
    for ch, sc in zip(chunks, schemes):
        if sc != 0:  # raw chunks are placed by the ingest pass, not by the decoders
            assert ob[pos:pos + len(ch)] == ch and orc[pos:pos + len(ch)] == ch, (len(ch), sc)
            assert opr[pos:pos + len(ch)] == ch, ("pair", len(ch), sc)
        pos += len(ch)
    assert pos == len(data)
    # corrupt the middle of the longest compressed chunk's stream
    big = max((e for e in idx if e[2] != 0), key=lambda e: e[1])
    bad = bytearray(body)
    mid = big[0] + 8 + big[1] // 2
    bad[mid:mid + 64] = bytes(rng.integers(0, 256, 64, dtype=np.uint8))
    ((ob, eb), (orc, er), (opr, epr)), _ = _decode_both(bytes(bad), chunks, len(chunks))
    assert eb == er == epr, (hex(eb), hex(er), hex(epr))
    if eb == 0:
        assert ob == orc == opr


def test_ingest_clip_window():
    data, ends, b = _make_runs("auto", seed=3)
    body = b.serialize(False)
    nck = len(ends)
    src = ops.padded_empty(len(body), DEV)
    src.copy_(torch.frombuffer(bytearray(body), dtype=torch.uint8))
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(body), 0, 0, nck, len(data))
    dst = ops.padded_empty(len(data), DEV)
    dst.zero_()
    hashes = torch.zeros((nck, 32), dtype=torch.uint8, device=DEV)
    lo, hi = 123_457, 987_653
    ops.ingest_terms(src, dst, terms, hashes, clip=(lo, hi))
    out = dst.cpu().numpy().tobytes()
    assert out[lo:hi] == data[lo:hi]
    assert out[:lo] == bytes(lo) and out[hi:] == bytes(len(data) - hi)
    # hashes are only meaningful for chunks entirely inside the clip window
    got = hashes.cpu().numpy()
    want = b.chunk_hashes()
    starts = [0] + ends[:-1]
    inside = [i for i, (a, e) in enumerate(zip(starts, ends)) if a >= lo and e <= hi]
    assert inside and all(got[i].tobytes() == want[i] for i in inside)


def test_clipped_ingests_on_two_streams():
    # Each workspace owns its clip scratch, so clipped decodes running concurrently on two streams
    # cannot overwrite each other's straddling chunks (they shared one global buffer before).
    data, ends, b = _make_runs("lz4", seed=11)
    body = b.serialize(False)
    nck = len(ends)
    src = ops.padded_empty(len(body), DEV)
    src.copy_(torch.frombuffer(bytearray(body), dtype=torch.uint8))
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(body), 0, 0, nck, len(data))
    windows = [(70_001, 650_003), (650_003, len(data) - 99_991)]
    dsts = [ops.padded_empty(len(data), DEV) for _ in windows]
    hashes = [torch.zeros((nck, 32), dtype=torch.uint8, device=DEV) for _ in windows]
    wss = [ops.IngestWorkspace(DEV, 1, nck) for _ in windows]
    streams = [torch.cuda.Stream(DEV) for _ in windows]
    for d in dsts:
        d.zero_()
    torch.cuda.synchronize()
    for _ in range(3):
        for d, h, ws, st, w in zip(dsts, hashes, wss, streams, windows):
            with torch.cuda.stream(st):
                ops.ingest_terms(src, d, terms, h, clip=w, ws=ws, check=False)
    torch.cuda.synchronize()
    for d, ws, (lo, hi) in zip(dsts, wss, windows):
        ops.raise_on_error(ws.err)
        out = d.cpu().numpy().tobytes()
        assert out[lo:hi] == data[lo:hi]
        assert out[:lo] == bytes(lo) and out[hi:] == bytes(len(data) - hi)
    # a clipped launch without scratch is refused instead of racing on shared memory
    H = ops.hip()
    with pytest.raises(RuntimeError):
        H.place_chunks(src.data_ptr(), len(body), dsts[0].data_ptr(), len(data), wss[0].chunks.data_ptr(), nck,
                       1, len(data), wss[0].err.data_ptr(), torch.cuda.current_stream().cuda_stream)


def test_ingest_detects_corruption():
    data, ends, b = _make_runs("auto", seed=5)
    body = bytearray(b.serialize(False))
    body[0] = 7  # bad header version
    src = ops.padded_empty(len(body), DEV)
    src.copy_(torch.frombuffer(body, dtype=torch.uint8))
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(body), 0, 0, len(ends), len(data))
    dst = ops.padded_empty(len(data), DEV)
    hashes = torch.zeros((len(ends), 32), dtype=torch.uint8, device=DEV)
    with pytest.raises(ops.IngestError):
        ops.ingest_terms(src, dst, terms, hashes)


def test_ingest_detects_bad_lz4_frame():
    data, ends, b = _make_runs("lz4", seed=6)
    body = bytearray(b.serialize(False))
    idx = C.index_chunks(bytes(body))
    comp = [e for e in idx if e[2] != 0]
    assert comp
    body[comp[len(comp) // 2][0] + 8] ^= 0xFF  # LZ4 frame magic of a compressed chunk
    src = ops.padded_empty(len(body), DEV)
    src.copy_(torch.frombuffer(body, dtype=torch.uint8))
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(body), 0, 0, len(ends), len(data))
    dst = ops.padded_empty(len(data), DEV)
    hashes = torch.zeros((len(ends), 32), dtype=torch.uint8, device=DEV)
    with pytest.raises(ops.IngestError):
        ops.ingest_terms(src, dst, terms, hashes)


def test_ingest_real_hf_xet_xorbs(tmp_path):
    hf_xet = pytest.importorskip("hf_xet")
    import glob
    import time
    files = []
    for name, d in (("bf", _bf16(500_000, 9)), ("txt", b"hello xet world " * 30_000)):
        f = tmp_path / name
        f.write_bytes(d)
        files.append(f)
    hf_xet.upload_files([str(f) for f in files], "local://" + str(tmp_path / "cas"),
                        ("t", int(time.time()) + 3600), None, None, "model")
    for x in glob.glob(str(tmp_path / "cas/xet/xorbs/xorbs/default.*")):
        blob = open(x, "rb").read()
        foot = C.parse_footer(blob)
        idx = C.index_chunks(blob)
        run = blob[:foot["footer_start"]]
        ulen = sum(e[3] for e in idx)
        src = ops.padded_empty(len(run), DEV)
        src.copy_(torch.frombuffer(bytearray(run), dtype=torch.uint8))
        dst = ops.padded_empty(ulen, DEV)
        terms = np.zeros(1, dtype=ops.TERM_DTYPE)
        terms[0] = (0, len(run), 0, 0, len(idx), ulen)
        hashes = torch.zeros((len(idx), 32), dtype=torch.uint8, device=DEV)
        ops.ingest_terms(src, dst, terms, hashes)
        assert [bytes(h) for h in hashes.cpu().numpy()] == foot["chunk_hashes"]
        want = C.extract_chunk_range(run, 0, len(idx))
        assert dst.cpu().numpy().tobytes() == want


@pytest.mark.parametrize("n", [1, 2, 3, 9, 10, 37, 1000, 20_000])
def test_merkle_matches_cpu(n):
    rng = np.random.default_rng(n)
    hs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sz = rng.integers(1, 131_072, size=n).astype(np.int64)
    leaves = [(hs[i].tobytes(), int(sz[i])) for i in range(n)]
    h_d = torch.from_numpy(hs).to(DEV)
    s_d = torch.from_numpy(sz).to(DEV)
    # two jobs: whole list + a sub-range
    jobs = [(0, n), (n // 3, n - n // 3)]
    roots = ops.merkle_roots(h_d, s_d, jobs, file_hash=True).cpu().numpy()
    assert roots[0].tobytes() == C.file_hash(leaves)
    assert roots[1].tobytes() == C.file_hash(leaves[n // 3:])
    raw = ops.merkle_roots(h_d, s_d, jobs[:1], file_hash=False).cpu().numpy()
    assert raw[0].tobytes() == C.merkle_root(leaves)


def test_merkle_large_sizes_and_many_jobs():
    """Sizes past 2^32 (the 64-bit decimal path), leaf and node sizes with 1..14 digits, and many
    small trees next to large ones (level-1 work spread over 8 workgroups per tree)."""
    rng = np.random.default_rng(99)
    n = 30_000
    hs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sz = (rng.integers(1, 10, size=n) * 10 ** rng.integers(0, 13, size=n)).astype(np.int64)
    sz[:50] = (1 << 32) + rng.integers(0, 1000, size=50)
    leaves = [(hs[i].tobytes(), int(sz[i])) for i in range(n)]
    h_d = torch.from_numpy(hs).to(DEV)
    s_d = torch.from_numpy(sz).to(DEV)
    jobs = [(0, n), (5, 1), (10, 2), (100, 17), (1000, 9000), (20_000, 10_000)] + [(i * 7, 7) for i in range(40)]
    roots = ops.merkle_roots(h_d, s_d, jobs, file_hash=True).cpu().numpy()
    for j, (b, m) in enumerate(jobs):
        assert roots[j].tobytes() == C.file_hash(leaves[b:b + m]), (b, m)


def test_cdc_candidates_match_cpu_chunker():
    rng = random.Random(11)
    data = rng.randbytes(3_000_000) + _bf16(500_000, 1) + bytes(200_000)
    t = ops.padded_empty(len(data), DEV)
    t.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    cand = ops.cdc_candidates(t)
    ends = ops.select_chunks(cand, len(data))
    assert list(map(int, ends)) == C.chunk_ends(data)


def test_cdc_candidates_misaligned_and_low_mask():
    """Candidate offsets at every buffer alignment and across segment edges, for the Xet mask (high
    word only) and a mask with low-word bits (the generic path), against the CPU oracle."""
    rng = random.Random(12)
    data = rng.randbytes(300_000)
    for off in (1, 3, 8, 15):
        t = ops.padded_empty(len(data) + off, DEV)
        t[off:].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
        for mask in (ops.XET_MASK, 0xF0000000000000F0):
            got = ops.cdc_candidates(t[off:], mask=mask)
            want = ops.cdc_candidates(t[off:].cpu(), mask=mask)
            assert got.tolist() == want.tolist(), (off, hex(mask))


def test_pack_chunks_matches_builder():
    rng = random.Random(4)
    data = rng.randbytes(900_000)
    ends = C.chunk_ends(data)
    b = C.XorbBuilder("none")
    prev = 0
    for e in ends:
        b.add_chunk(data[prev:e])
        prev = e
    body = b.serialize(False)
    starts = np.array([0] + ends[:-1], dtype=np.uint64)
    lens = np.diff(np.array([0] + ends, dtype=np.uint64)).astype(np.uint32)
    out_off = np.array([0] + b.chunk_boundaries()[:-1], dtype=np.uint64) + 5
    d = ops.padded_empty(len(data) + 3, DEV)
    d[3:].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    out = ops.padded_empty(len(body) + 5, DEV)
    out.zero_()
    ops.pack_chunks(d, starts + 3, lens, out_off, out)
    assert out.cpu().numpy().tobytes()[5:] == body


def test_fill_synthetic_deterministic():
    a = ops.padded_empty(1 << 20, DEV)
    b = ops.padded_empty((1 << 20) + 5, DEV)
    ops.fill_synthetic(a, 42, 0, 0)
    ops.fill_synthetic(b[5:], 42, 0, 0)  # different dst alignment, same stream
    assert torch.equal(a, b[5:5 + (1 << 20)])
    c = ops.padded_empty(1000, DEV)
    ops.fill_synthetic(c, 42, 12345, 0)  # stream offset selects the same bytes
    assert torch.equal(c, a[12345:13345])
    f = ops.padded_empty(1 << 20, DEV)
    ops.fill_synthetic(f, 7, 0, 1)
    v = f.view(torch.bfloat16).float()
    assert abs(v.std().item() - 0.02) < 0.002 and abs(v.mean().item()) < 0.002


def test_sha1_info_hash_kernel():
    import hashlib

    g = torch.Generator().manual_seed(3)
    hs = torch.randint(0, 256, (1000, 32), dtype=torch.uint8, generator=g)
    got = ops.sha1_info_hash(hs.cuda()).cpu().numpy()
    for i in range(0, 1000, 37):
        assert got[i].tobytes() == hashlib.sha1(b"zest-xet-v1:" + hs[i].numpy().tobytes()).digest()
    assert ops.sha1_info_hash(hs[:0].cuda()).shape == (0, 20)


def test_gpu_lz4_compress_roundtrip_host_decoder():
    """K7b: GPU BG4/LZ4 frames decode with the host decoder (same frame format as hf_xet) to the
    original bytes; incompressible chunks are reported as raw; ratios close to the host encoder."""
    from zest_amd import _core, ops
    rng = np.random.default_rng(5)
    w = (rng.standard_normal(300_000).astype(np.float32) * 0.02)
    bf16 = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
    parts = [bf16[:65536], bf16[65536:65536 + 131072], rng.integers(0, 8, 70_000, dtype=np.uint8).tobytes(),
             rng.integers(0, 256, 50_000, dtype=np.uint8).tobytes(), bytes(40_000), b"abc" * 9, b"x" * 12,
             bf16[200_000:200_000 + 8191]]
    blob = b"".join(parts)
    offs = np.cumsum([0] + [len(p) for p in parts[:-1]]).astype(np.uint64)
    lens = np.array([len(p) for p in parts], dtype=np.uint32)
    dev = torch.device("cuda:0")
    buf = ops.padded_empty(len(blob), dev)
    buf.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    for bg4, scheme in ((True, 2), (False, 1)):
        frames, flen = ops.compress_chunks(buf, offs, lens, bg4=bg4)
        host = frames.cpu().numpy()
        gpu_total = host_total = 0
        for i, p in enumerate(parts):
            if flen[i] == 0:
                assert len(p) < 64 or len(_core.compress_chunk(p, "bg4" if bg4 else "lz4")[1]) >= len(p) * 0.95, i
                gpu_total += len(p)
            else:
                fr = host[i * ops.LZ4_SLOT:i * ops.LZ4_SLOT + int(flen[i])].tobytes()
                assert _core.decompress_chunk(scheme, fr, len(p)) == p, (bg4, i)
                gpu_total += int(flen[i])
            host_total += min(len(p), len(_core.compress_chunk(p, "bg4" if bg4 else "lz4")[1]))
        assert gpu_total <= host_total * 1.15, (bg4, gpu_total, host_total)


def test_gpu_lz4_compress_staged_matches_v1(monkeypatch):
    """The default compressor (4-byte tagged table, LDS-staged output) writes exactly the frames of
    the v1 kernel (8-byte table, direct stores): same hits, same parse, byte-identical frames,
    across bf16 / low-entropy / random / zero / tiny / 128 KiB chunks and long literal runs."""
    rng = np.random.default_rng(8)
    w = (rng.standard_normal(600_000).astype(np.float32) * 0.02)
    bf16 = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
    parts = [bf16[:65536], bf16[65536:65536 + 131072], rng.integers(0, 8, 70_000, dtype=np.uint8).tobytes(),
             rng.integers(0, 256, 50_000, dtype=np.uint8).tobytes(), bytes(131072), b"abc" * 9, b"x" * 12,
             bf16[300_000:300_000 + 8191], rng.integers(0, 256, 3000, dtype=np.uint8).tobytes() * 20,
             rng.integers(0, 256, 40_000, dtype=np.uint8).tobytes() + bytes(20_000)]
    parts += [bf16[i * 70_000:i * 70_000 + 70_000] for i in range(8)]
    blob = b"".join(parts)
    offs = np.cumsum([0] + [len(p) for p in parts[:-1]]).astype(np.uint64)
    lens = np.array([len(p) for p in parts], dtype=np.uint32)
    buf = ops.padded_empty(len(blob), DEV)
    buf.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    for bg4 in (True, False):
        monkeypatch.delenv("ZG_COMPRESS", raising=False)
        f2, l2 = ops.compress_chunks(buf, offs, lens, bg4=bg4)
        monkeypatch.setenv("ZG_COMPRESS", "v1")
        f1, l1 = ops.compress_chunks(buf, offs, lens, bg4=bg4)
        assert np.array_equal(l1, l2), (bg4, l1, l2)
        h1, h2 = f1.cpu().numpy(), f2.cpu().numpy()
        for i in range(len(parts)):
            a = i * ops.LZ4_SLOT
            assert np.array_equal(h1[a:a + int(l1[i])], h2[a:a + int(l2[i])]), (bg4, i)
            if l2[i]:
                fr = h2[a:a + int(l2[i])].tobytes()
                assert C.decompress_chunk(2 if bg4 else 1, fr, len(parts[i])) == parts[i], (bg4, i)
    monkeypatch.delenv("ZG_COMPRESS", raising=False)


def test_gpu_pull_of_bg4_compressed_world():
    """End to end on the decode path: a bf16 world whose chunks are BG4-LZ4 frames compressed on
    the GPU (as Xet stores checkpoints) is pulled by the device engine (header walk -> LZ4/BG4 decode
    -> BLAKE3 -> Merkle) and lands byte-exact."""
    from zest_amd import ops
    from zest_amd.engine import DevicePuller
    from zest_amd.synthetic import SyntheticWorld
    dev = torch.device("cuda:0")
    w = SyntheticWorld("llama-tiny", seed=9, mode="bf16", max_xorb_bytes=1 << 20, compression="bg4")
    arena = ops.padded_empty(w.arena_bytes, dev)
    w.generate_on_device(arena)
    w.build_on_device(arena)
    assert (w.chunk_scheme == 2).mean() > 0.9 and w.chunk_clen.sum() < 0.95 * w.chunk_len.sum()
    want = arena.clone()
    p = DevicePuller(w, arena, 0, 1, round_bytes=1 << 20)
    p.build_origin()
    assert p.origin.n == int(w.chunk_clen.sum()) + 8 * w.n_chunks
    for _ in range(2):
        arena.fill_(0)
        p.err.zero_()
        p.step()
        torch.cuda.synchronize()
        p.check()
        for f in w.xet_files:  # (the alignment gaps between files are not part of the repository)
            assert torch.equal(arena[f.arena_off:f.arena_off + f.size], want[f.arena_off:f.arena_off + f.size]), f.path
    # back-to-back steps without a host sync: the host stays at most `steps_ahead` steps ahead
    for _ in range(6):
        p.step()
        assert len(p._inflight) <= p.steps_ahead + 1
    torch.cuda.synchronize()
    p.check()
    p.close()


def test_build_ser_store_is_the_origin():
    """A compressed build with ser_store writes every chunk serialized in chunk order; a one-rank
    DevicePuller adopts it as its origin (build_origin is then a no-op) and the bytes equal the
    origin build_origin makes by compressing again; the pull from it is byte-exact."""
    from zest_amd.engine import DevicePuller, pinned_take
    from zest_amd.synthetic import SyntheticWorld
    dev = torch.device("cuda:0")
    w = SyntheticWorld("llama-tiny", seed=9, mode="bf16", max_xorb_bytes=1 << 20, compression="bg4")
    arena = ops.padded_empty(w.arena_bytes, dev)
    w.generate_on_device(arena)
    cap, ptr = pinned_take(int(w.model_bytes * 1.002) + (16 << 20))
    w.build_on_device(arena, ser_store=(ptr, cap))
    assert w.serialized is not None and w.serialized[2] == int(w.chunk_clen.sum()) + 8 * w.n_chunks
    want = arena.clone()
    ref = DevicePuller(w, arena, 0, 1, round_bytes=1 << 20)  # adopts the store
    assert ref.origin_prebuilt and ref.origin.ptr == ptr and w.serialized is None
    adopted = ref.origin.array[:ref.origin.n].copy()
    ref.origin_prebuilt = False
    ref.origin.array[:] = 0
    ref.build_origin()  # the old path: compress every chunk again and pack
    torch.cuda.synchronize()
    assert np.array_equal(ref.origin.array[:ref.origin.n], adopted)
    for _ in range(2):
        arena.fill_(0)
        ref.err.zero_()
        ref.step()
        torch.cuda.synchronize()
        ref.check()
        for f in w.xet_files:
            assert torch.equal(arena[f.arena_off:f.arena_off + f.size], want[f.arena_off:f.arena_off + f.size]), f.path
    # a ser_store too small for the build fails loudly (before any byte is copied into it)
    w2 = SyntheticWorld("llama-tiny", seed=9, mode="bf16", max_xorb_bytes=1 << 20, compression="bg4")
    with pytest.raises(RuntimeError, match="ser_store too small"):
        w2.build_on_device(arena, ser_store=(ptr, 1 << 16))
    ref.close()  # the adopted buffer goes back to the pinned pool


@pytest.mark.parametrize("compression", ["none", "bg4"])
def test_device_puller_hip_graph_replay(compression):
    """A whole one-GPU step captured into a HIP graph and replayed: byte-exact arena, the Merkle
    check still runs every replay (a corrupted origin byte is caught on the next replay)."""
    from zest_amd import ops
    from zest_amd.engine import DevicePuller
    from zest_amd.synthetic import SyntheticWorld
    dev = torch.device("cuda:0")
    w = SyntheticWorld("llama-tiny", seed=10, mode="bf16", max_xorb_bytes=256 << 10, compression=compression)
    arena = ops.padded_empty(w.arena_bytes, dev)
    w.generate_on_device(arena)
    w.build_on_device(arena)
    want = arena.clone()
    p = DevicePuller(w, arena, 0, 1, round_bytes=256 << 10)  # > 4 rounds: tapered, slots reused
    assert p.n_rounds > p.slots + 2
    p.build_origin()
    assert p.capture_graph()
    for _ in range(3):
        arena.fill_(0xA5)
        p.err.zero_()
        p.step()
        torch.cuda.synchronize()
        p.check()
        for f in w.xet_files:
            assert torch.equal(arena[f.arena_off:f.arena_off + f.size], want[f.arena_off:f.arena_off + f.size]), f.path
    # the replayed graph reads the live origin: flip one payload byte there and the check fails
    p.origin.array[p.origin.n // 2] ^= 0x40
    p.err.zero_()
    p.step()
    torch.cuda.synchronize()
    with pytest.raises(ops.IngestError):
        p.check()
    p.close()


def test_device_puller_host_header_walk_matches_device_walk():
    """The engine's host header walk (default) and the device walk (ZEST_HOST_INDEX=0) give the
    same byte-exact pull; a corrupted chunk header in the origin is reported by the host walk."""
    import os

    from zest_amd import ops
    from zest_amd.engine import DevicePuller
    from zest_amd.synthetic import SyntheticWorld
    dev = torch.device("cuda:0")
    w = SyntheticWorld("llama-tiny", seed=12, mode="bf16", max_xorb_bytes=256 << 10, compression="bg4")
    arena = ops.padded_empty(w.arena_bytes, dev)
    w.generate_on_device(arena)
    w.build_on_device(arena)
    want = arena.clone()
    pullers = []
    for host in ("1", "0"):
        # the host walk runs in the "lanes" pipeline (a compressed world defaults to "copy", which
        # keeps the device walk)
        os.environ.update(ZEST_HOST_INDEX=host, ZEST_PIPELINE="lanes")
        try:
            p = DevicePuller(w, arena, 0, 1, round_bytes=256 << 10)
        finally:
            os.environ.pop("ZEST_HOST_INDEX", None)
            os.environ.pop("ZEST_PIPELINE", None)
        assert p.host_index == (host == "1") and p.pipeline == "lanes"
        p.build_origin()
        for _ in range(3):  # both parities of the host record tables
            arena.fill_(0x5A)
            p.err.zero_()
            p.step()
            torch.cuda.synchronize()
            p.check()
            for f in w.xet_files:
                assert torch.equal(arena[f.arena_off:f.arena_off + f.size], want[f.arena_off:f.arena_off + f.size])
        pullers.append(p)
    p = pullers[0]
    p.origin.array[0] = 7  # version byte of the first chunk header of the first term
    p.err.zero_()
    p.step()
    torch.cuda.synchronize()
    with pytest.raises(ops.IngestError) as ei:
        p.check()
    assert ei.value.code == 1
    for q in pullers:
        q.close()


@pytest.mark.parametrize("pipeline", ["copy", "lanes"])
@pytest.mark.parametrize("mode,compression", [("bf16", "bg4"), ("random", "none")])
def test_device_puller_pipelines(pipeline, mode, compression):
    """Both engine pipeline shapes ("copy": one H2D stream gated by slot events, the default for
    compressed worlds; "lanes": H2D on the compute lanes, the default for raw ones) pull every byte
    exactly over several steps."""
    import os

    from zest_amd import ops
    from zest_amd.engine import DevicePuller
    from zest_amd.synthetic import SyntheticWorld
    dev = torch.device("cuda:0")
    w = SyntheticWorld("llama-tiny", seed=13, mode=mode, max_xorb_bytes=256 << 10, compression=compression)
    arena = ops.padded_empty(w.arena_bytes, dev)
    w.generate_on_device(arena)
    w.build_on_device(arena)
    want = arena.clone()
    os.environ.update(ZEST_PIPELINE=pipeline)
    try:
        p = DevicePuller(w, arena, 0, 1, round_bytes=256 << 10, slots=4)
    finally:
        os.environ.pop("ZEST_PIPELINE", None)
    assert p.pipeline == pipeline and p.n_rounds >= 4
    p.build_origin()
    for _ in range(3):
        arena.fill_(0x3C)
        p.err.zero_()
        p.step()
    torch.cuda.synchronize()
    p.check()
    for f in w.xet_files:  # (the arena also holds alignment gaps that belong to no file)
        assert torch.equal(arena[f.arena_off:f.arena_off + f.size], want[f.arena_off:f.arena_off + f.size])


FELL_BACK = 1 << 31  # k_hdr_link's mark in the scan's per-term candidate counts


def _index_both(src, terms, n_chunks, fallbacks=None):
    """Chunk records + error word of the serial header walk and of the parallel scan/link walk;
    `fallbacks` (a list) receives, per term, whether the link handed it to the serial walk."""
    H = ops.hip()
    st = torch.cuda.current_stream().cuda_stream
    tdev = torch.from_numpy(terms.view(np.uint8).copy()).to(DEV)
    out = []
    for scan in (False, True):
        chunks = torch.zeros(max(1, n_chunks) * ops.CHUNK_DTYPE.itemsize, dtype=torch.uint8, device=DEV)
        err = torch.zeros(1, dtype=torch.int64, device=DEV)
        if scan:
            sb = H.index_scratch_bytes(len(terms))
            scr = torch.empty(sb, dtype=torch.uint8, device=DEV)
            H.index_terms_scan(src.data_ptr(), src.numel(), tdev.data_ptr(), len(terms), chunks.data_ptr(),
                               err.data_ptr(), scr.data_ptr(), sb, st)
        else:
            H.index_terms(src.data_ptr(), tdev.data_ptr(), len(terms), chunks.data_ptr(), err.data_ptr(), st)
        torch.cuda.synchronize()
        out.append((chunks.cpu().numpy().tobytes(), int(err.item())))
        if scan and fallbacks is not None:
            cnt = scr[:4 * len(terms)].cpu().numpy().view(np.uint32)
            fallbacks[:] = [bool(int(c) & FELL_BACK) for c in cnt]
    return out


@pytest.mark.parametrize("policy", ["none", "bg4", "auto"])
def test_index_scan_matches_serial_walk(policy):
    """K4 parallel header walk (candidate scan + LDS sort/link + prefix sum) gives byte-identical
    chunk records to the serial walk: clean runs at odd offsets (no term falls back); a raw chunk
    carrying a planted header-like pattern (a false candidate: the link picks the chain around it,
    no fallback); two planted look-alikes where the first points at the second (an ambiguous set:
    that term falls back to the serial walk); and a corrupted header (same error word)."""
    data, ends, b = _make_runs(policy, seed=3)
    body = b.serialize(False)
    nck = len(ends)
    bounds = b.chunk_boundaries()
    cuts = [0, nck // 4, nck // 2, 3 * nck // 4, nck]
    uoffs = [0] + list(ends)
    src_host = bytearray(17)
    terms = np.zeros(4, dtype=ops.TERM_DTYPE)
    for t in range(4):
        c0, c1 = cuts[t], cuts[t + 1]
        r0 = 0 if c0 == 0 else bounds[c0 - 1]
        run = body[r0:bounds[c1 - 1]]
        terms[t] = (len(src_host), len(run), 5 + uoffs[c0], c0, c1 - c0, uoffs[c1] - uoffs[c0])
        src_host += run + b"\x07" * (t + 1)
    src = ops.padded_empty(len(src_host), DEV)
    src.copy_(torch.frombuffer(bytes(src_host), dtype=torch.uint8))
    fb = []
    (serial, e0), (scan, e1) = _index_both(src, terms, nck, fb)
    assert e0 == 0 and e1 == 0 and scan == serial
    assert fb == [False] * 4, fb
    # the records are the real ones: ingest through them reproduces the data
    if policy == "none":
        # a planted plausible header (version 0, raw, clen == ulen == 16) inside term 1's first payload
        t = 1
        pos = int(terms[t]["src"]) + 8 + 100
        src_host[pos:pos + 8] = bytes([0, 16, 0, 0, 0, 16, 0, 0])
        src.copy_(torch.frombuffer(bytes(src_host), dtype=torch.uint8))
        (serial, e0), (scan, e1) = _index_both(src, terms, nck, fb)
        assert e0 == 0 and e1 == 0 and scan == serial
        assert fb == [False] * 4, fb
        # term 3: look-alike A (clen 16) whose successor is look-alike B (clen 24): B is some
        # candidate's successor, so the chosen set has one member too many -> the serial walk
        t = 3
        pa = int(terms[t]["src"]) + 8 + 200
        pb = pa + 8 + 16
        src_host[pa:pa + 8] = bytes([0, 16, 0, 0, 0, 16, 0, 0])
        src_host[pb:pb + 8] = bytes([0, 24, 0, 0, 0, 24, 0, 0])
        # ...and B's successor is a real header (the chunk after the first one), so B passes the
        # successor test: only the member count can reject the set
        first = int(bounds[int(terms[t]["chunk_base"])]) - (0 if int(terms[t]["chunk_base"]) == 0
                                                           else int(bounds[int(terms[t]["chunk_base"]) - 1]))
        nxt = int(terms[t]["src"]) + first
        if nxt - (pb + 8) > 0 and nxt - (pb + 8) < (1 << 17):
            cl = nxt - (pb + 8)
            src_host[pb:pb + 8] = bytes([0, cl & 0xFF, (cl >> 8) & 0xFF, cl >> 16, 0, cl & 0xFF, (cl >> 8) & 0xFF, cl >> 16])
        src.copy_(torch.frombuffer(bytes(src_host), dtype=torch.uint8))
        (serial, e0), (scan, e1) = _index_both(src, terms, nck, fb)
        assert e0 == 0 and e1 == 0 and scan == serial
        assert fb == [False, False, False, True], fb
    # a corrupted header in term 2: both walks report the same error and the same zeroed records
    pos = int(terms[2]["src"])
    src_host[pos + 4] = 9
    src.copy_(torch.frombuffer(bytes(src_host), dtype=torch.uint8))
    (serial, e0), (scan, e1) = _index_both(src, terms, nck)
    assert e0 != 0 and e1 == e0 and scan == serial


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_index_scan_random_lookalikes(seed):
    """The parallel walk against the serial walk with header look-alikes planted at random payload
    positions: lone ones (the link must see past them), chains of two, and ones whose successor is a
    real header (both kinds make the chosen set ambiguous -> that term falls back).  Records and the
    error word must equal the serial walk's whatever path each term took."""
    rng = random.Random(seed)
    data, ends, b = _make_runs("none" if seed % 2 else "auto", seed=seed)
    body = b.serialize(False)
    nck = len(ends)
    bounds = list(b.chunk_boundaries())
    cuts = [0, nck // 3, 2 * nck // 3, nck]
    uoffs = [0] + list(ends)
    src_host = bytearray(3)
    terms = np.zeros(3, dtype=ops.TERM_DTYPE)
    for t in range(3):
        c0, c1 = cuts[t], cuts[t + 1]
        r0 = 0 if c0 == 0 else bounds[c0 - 1]
        terms[t] = (len(src_host), bounds[c1 - 1] - r0, uoffs[c0], c0, c1 - c0, uoffs[c1] - uoffs[c0])
        src_host += body[r0:bounds[c1 - 1]] + b"\x00" * 5
    hdr_pos = {int(terms[t]["src"]) + (0 if c == cuts[t] else bounds[c - 1] - (0 if cuts[t] == 0 else bounds[cuts[t] - 1]))
               for t in range(3) for c in range(cuts[t], cuts[t + 1])}

    def raw_hdr(n):
        return bytes([0, n & 0xFF, (n >> 8) & 0xFF, n >> 16, 0, n & 0xFF, (n >> 8) & 0xFF, n >> 16])

    def plant(pos, n):  # only inside payloads, never over a real header
        if any(h - 8 < pos < h + 8 for h in hdr_pos):
            return False
        src_host[pos:pos + 8] = raw_hdr(n)
        return True

    for _ in range(rng.randint(1, 6)):
        t = rng.randrange(3)
        lo = int(terms[t]["src"]) + 16
        pos = rng.randrange(lo, lo + int(terms[t]["src_len"]) - 64)
        kind = rng.randrange(3)
        if kind == 0:  # lone look-alike
            plant(pos, rng.randint(1, 4096))
        elif kind == 1:  # a chain of two
            n1 = rng.randint(1, 512)
            if plant(pos, n1):
                plant(pos + 8 + n1, rng.randint(1, 512))
        else:  # a look-alike whose successor is the next real header
            nxt = min((h for h in hdr_pos if h > pos + 16), default=None)
            if nxt is not None and nxt - pos - 8 <= 131072:
                plant(pos, nxt - pos - 8)
    src = ops.padded_empty(len(src_host), DEV)
    src.copy_(torch.frombuffer(bytes(src_host), dtype=torch.uint8))
    fb = []
    (serial, e0), (scan, e1) = _index_both(src, terms, nck, fb)
    assert e0 == 0 and e1 == e0 and scan == serial, (fb, e0, e1)


@pytest.mark.gpu
def test_ingest_many_small_bg4_chunks_dynamic_schedule(monkeypatch):
    """More chunks than decoder blocks (4096): under the dynamic schedule every block takes chunk
    after chunk from the work counter (LDS ticket ring between its producer and consumer waves),
    interleaved with stored chunks the producer settles itself; bytes and hashes equal the host
    builder's, and the static schedule's."""
    rng = np.random.default_rng(11)
    b = C.XorbBuilder("auto")
    parts = []
    for i in range(5000):
        n = int(rng.integers(600, 2600))
        if i % 7 == 3:
            p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()  # incompressible: stored
        else:
            w = rng.standard_normal(n // 2).astype(np.float32) * 0.02
            p = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
        assert b.fits(len(p))
        b.add_chunk(p)
        parts.append(p)
    data = b"".join(parts)
    body = b.serialize(False)
    nck = len(parts)
    H = ops.hip()
    src = ops.padded_empty(len(body), DEV)
    src.copy_(torch.frombuffer(bytearray(body), dtype=torch.uint8))
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(body), 0, 0, nck, len(data))
    ws = ops.IngestWorkspace(DEV, 1, nck)
    terms_d = torch.from_numpy(terms.view(np.uint8).copy()).to(DEV)
    ops.index_terms(H, src.data_ptr(), len(body), terms_d.data_ptr(), 1, ws.chunks.data_ptr(), ws.err.data_ptr(),
                    torch.cuda.current_stream().cuda_stream, ws)
    torch.cuda.synchronize()
    rec = np.frombuffer(ws.chunks[: nck * ops.CHUNK_DTYPE.itemsize].cpu().numpy().tobytes(), dtype=ops.CHUNK_DTYPE)
    assert (rec["scheme"] != 0).sum() > 4096 and (rec["scheme"] == 0).any()
    got = {}
    for dyn in ("1", "0"):
        monkeypatch.setenv("ZG_PAIR_DYNAMIC", dyn)
        dst = ops.padded_empty(len(data), DEV)
        dst.fill_(0x3C)
        hashes = torch.full((nck, 32), 0x77, dtype=torch.uint8, device=DEV)
        err = torch.zeros(1, dtype=torch.int64, device=DEV)
        sp, sb = ops.HashScratch(DEV, ingest=True).get(nck, len(data))
        H.ingest_chunks(src.data_ptr(), len(body), dst.data_ptr(), len(data), ws.chunks.data_ptr(), nck, True,
                        err.data_ptr(), hashes.data_ptr(), 0, 0, torch.cuda.current_stream().cuda_stream, sp, sb)
        torch.cuda.synchronize()
        assert int(err.item()) == 0, dyn
        assert dst.cpu().numpy().tobytes() == data, dyn
        got[dyn] = hashes.cpu().numpy()
    monkeypatch.delenv("ZG_PAIR_DYNAMIC")
    assert np.array_equal(got["1"], got["0"])
    assert got["1"].tobytes() == b"".join(b.chunk_hashes())
