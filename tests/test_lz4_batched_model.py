"""Executable model of the batched LZ4 decoder's algorithm (csrc/gpu/lz4seq.hip), run on the CPU.

The kernel splits LZ4 into a serial parse (sequences -> 64-record batches) and a lane-parallel
execute: literal bytes, then match bytes, 64 per pass, each match byte reading its periodic
source `start - off + k % off`, with sources written by the same pass chased to the writer's own
source, and near sources (< kRing behind the batch end) read from a per-wave history ring that only
short batches may trust.  This file re-implements exactly those rules with numpy "lanes" and checks
the result against the host LZ4 decoder on frames from the host encoder, so the algorithm (not just
one GPU run) is pinned: every data shape the GPU tests use plus RLE runs, long literal runs, far
repeats and overlapping short offsets.
"""
from __future__ import annotations

import struct

import numpy as np
import pytest

from zest_amd import _core as C

WAVE = 64
RING = 4096


def parse_frame(frame: bytes):
    """LZ4 frame -> list of (literal_pos, literal_len, match_len, offset) records, literal runs split
    at 0xFFFF and matches at 0x7FFF exactly like the kernel's emit()."""
    assert struct.unpack_from("<I", frame, 0)[0] == 0x184D2204
    flg = frame[4]
    ip = 7 + (8 if flg & 8 else 0) + (4 if flg & 1 else 0)
    bck = 4 if flg & 0x10 else 0
    recs = []

    def emit(lp, lit, ml, off):
        while lit > 0xFFFF:
            recs.append((lp, 0xFFFF, 0, 0))
            lp += 0xFFFF
            lit -= 0xFFFF
        first = True
        while first or ml:
            m = min(ml, 0x7FFF)
            recs.append((lp, lit, m, off if m else 0))
            lp += lit
            lit = 0
            ml -= m
            first = False

    while True:
        bs = struct.unpack_from("<I", frame, ip)[0]
        ip += 4
        if bs == 0:
            break
        ln = bs & 0x7FFFFFFF
        if bs >> 31:
            emit(ip, ln, 0, 0)
            ip += ln
        else:
            bend = ip + ln
            while True:
                tok = frame[ip]
                ip += 1
                lit = tok >> 4
                if lit == 15:
                    while True:
                        b = frame[ip]
                        ip += 1
                        lit += b
                        if b != 255:
                            break
                lp = ip
                ip += lit
                if ip == bend:
                    emit(lp, lit, 0, 0)
                    break
                off = frame[ip] | (frame[ip + 1] << 8)
                ip += 2
                ml = tok & 15
                if ml == 15:
                    while True:
                        b = frame[ip]
                        ip += 1
                        ml += b
                        if b != 255:
                            break
                emit(lp, lit, ml + 4, off)
        ip += bck
    return recs


def model_decode(frame: bytes, ulen: int, batch: int = WAVE) -> bytes:
    recs = parse_frame(frame)
    out = np.full(ulen, -1, dtype=np.int64)       # HBM (what stores have produced so far)
    ring = np.full(RING, -1, dtype=np.int64)      # the wave's LDS history
    src = np.frombuffer(frame, dtype=np.uint8)
    obase = 0
    for b0 in range(0, len(recs), batch):         # the kernel executes 59..64 records at a time
        batch_recs = recs[b0:b0 + batch]
        lit = np.array([r[1] for r in batch_recs], dtype=np.int64)
        ml = np.array([r[2] for r in batch_recs], dtype=np.int64)
        off = np.array([r[3] for r in batch_recs], dtype=np.int64)
        lpos = np.array([r[0] for r in batch_recs], dtype=np.int64)
        opos = obase + np.cumsum(lit + ml) - lit - ml
        mstart = opos + lit
        span = int((lit + ml).sum())
        oend = obase + span
        # literal phase (byte t of the batch's literal bytes on lane t % 64)
        li = np.cumsum(lit)
        for t in range(int(li[-1]) if len(li) else 0):
            s = int(np.searchsorted(li, t, side="right"))
            k = t - (li[s] - lit[s])
            p = opos[s] + k
            out[p] = ring[p % RING] = src[lpos[s] + k]
        # match passes
        mi = np.cumsum(ml)
        mtot = int(mi[-1]) if len(mi) else 0
        short = span + 4 * WAVE < RING
        for t0 in range(0, mtot, WAVE):
            t = np.arange(t0, min(t0 + WAVE, mtot))
            s = np.searchsorted(mi, t, side="right")
            k = t - (mi[s] - ml[s])
            o = np.maximum(off[s], 1)
            d = mstart[s] + k
            q = mstart[s] - o + k % o
            while True:  # chase sources written by this same pass
                j = np.searchsorted(d, q)
                pend = (j < len(d)) & (d[np.minimum(j, len(d) - 1)] == q)
                if not pend.any():
                    break
                q = np.where(pend, q[np.minimum(j, len(d) - 1)], q)
            if short:
                far = oend - q >= RING
                v = np.where(far, out[q], ring[q % RING])
            else:
                v = out[q]          # long batch: HBM read-back after s_waitcnt
            assert (v >= 0).all(), "read a byte before it was written"
            out[d] = v
            ring[d % RING] = v
        if not short:               # rebuild the ring from HBM
            lo = max(0, oend - RING)
            ring[np.arange(lo, oend) % RING] = out[lo:oend]
        obase = oend
    assert obase == ulen and (out >= 0).all()
    return out.astype(np.uint8).tobytes()


def _bf16(n, seed):
    w = np.random.default_rng(seed).standard_normal(n // 2).astype(np.float32) * 0.02
    return (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()


def _cases():
    rng = np.random.default_rng(3)
    phrase = rng.integers(0, 256, 3000, dtype=np.uint8)
    far = np.resize(phrase, 60_000).copy()
    far[rng.integers(0, far.size, 500)] = rng.integers(0, 256, 500, dtype=np.uint8)
    return {
        "bf16": _bf16(65_536, 1),
        "bf16_128k": _bf16(131_072, 2),
        "zeros": bytes(131_072),
        "rle_short_offsets": (b"ab" * 9000 + b"xyz" * 7000 + b"q" * 20_000),
        "long_literals_then_repeats": rng.integers(0, 256, 40_000, dtype=np.uint8).tobytes() + b"hello " * 4000,
        "lowent": (rng.integers(0, 8, 65_536, dtype=np.uint8) * 31).tobytes(),
        "far_repeats": far.tobytes(),
        "text": b"zest xorb ingest test line. " * 2500,
        "sparse": np.where(rng.random(65_536) < 0.02, rng.integers(0, 256, 65_536), 0).astype(np.uint8).tobytes(),
    }


@pytest.mark.parametrize("policy", ["lz4", "bg4"])
@pytest.mark.parametrize("name", sorted(_cases()))
def test_batched_decode_model_matches_host_decoder(name, policy):
    data = _cases()[name]
    scheme, frame = C.compress_chunk(data, policy)
    if scheme == 0:
        pytest.skip("stored uncompressed")
    grouped = C.decompress_chunk(1, frame, len(data))  # the LZ4 stream's own output (BG4: grouped)
    for batch in (64, 59, 37):
        assert model_decode(frame, len(data), batch) == grouped, batch
    assert C.decompress_chunk(scheme, frame, len(data)) == data
