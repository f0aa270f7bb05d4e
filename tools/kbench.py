#!/usr/bin/env python3
"""Kernel micro-benchmarks on one MI355X: throughput of every HIP kernel in zest_amd.ops.

Prints one JSON line per kernel: {"kernel", "gbps", "ms", "bytes", ...}.  Uses HIP events around
`--iters` back-to-back launches after a warm-up; data is random (not zero-filled).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
if os.environ.get("ZEST_PKG_ROOT"):  # A/B of kernel builds: a package copy with another _hip .so
    sys.path.insert(0, os.environ["ZEST_PKG_ROOT"])

from zest_amd import _core as C
from zest_amd import ops


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = int(a.gib * (1 << 30))
    sel = set(a.only.split(",")) if a.only else None

    def want(k):
        return sel is None or k in sel

    H = ops.hip()
    st = torch.cuda.current_stream().cuda_stream
    arena = ops.padded_empty(n, dev)
    ops.fill_synthetic(arena, 1, 0, 0)
    torch.cuda.synchronize()

    if want("fill"):
        ms = timed(lambda: ops.fill_synthetic(arena, 1, 0, 0), a.iters)
        emit(kernel="fill_synthetic_random", bytes=n, ms=ms, gbps=n / ms / 1e6)

    # fixed 64 KiB chunks over the arena
    csize = 65536
    nck = n // csize
    offs = np.arange(nck, dtype=np.uint64) * csize
    lens = np.full(nck, csize, dtype=np.uint32)
    offs_d = torch.from_numpy(offs.view(np.int64)).to(dev)
    lens_d = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty((nck, 32), dtype=torch.uint8, device=dev)
    hs = ops.HashScratch(dev)

    def hash_case(name, o, ln, check_n=4):
        """K1 over (offset, len) messages: wave-per-message kernel vs the leaf-flat pipeline."""
        o_d = torch.from_numpy(o.astype(np.int64)).to(dev)
        l_d = torch.from_numpy(ln.astype(np.uint32).view(np.int32)).to(dev)
        m = len(o)
        res = torch.empty((m, 32), dtype=torch.uint8, device=dev)
        nb = int(ln.sum())
        sp, sb = hs.get(m, nb)
        for path, scr in (("wave", (0, 0)), ("flat", (sp, sb))):
            ms = timed(lambda: H.hash_ranges(arena.data_ptr(), o_d.data_ptr(), l_d.data_ptr(), m, res.data_ptr(), 0,
                                             st, *scr), a.iters)
            emit(kernel=f"blake3_{name}[{path}]", bytes=nb, ms=ms, gbps=nb / ms / 1e6, chunks=m)
            h = res[:check_n].cpu().numpy()
            host = arena[: int(o[check_n - 1] + ln[check_n - 1])].cpu().numpy().tobytes()
            assert all(h[i].tobytes() == C.chunk_hash(host[int(o[i]):int(o[i]) + int(ln[i])]) for i in range(check_n))

    if want("hash"):
        hash_case("xet_chunks_64k", offs, lens)
        # CDC chunks land at arbitrary byte offsets in the arena: the misaligned load path
        hash_case("xet_chunks_64k_unaligned", offs + (np.arange(nck, dtype=np.uint64) * 13) % 61,
                  np.full(nck, csize - 64, dtype=np.uint32))
        # the real size mix: Xet CDC chunks (8-128 KiB) of the arena's own bytes
        ends = np.asarray(C.chunk_ends(arena[: min(n, 256 << 20)].cpu().numpy().tobytes()), dtype=np.uint64)
        starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64)
        hash_case("xet_chunks_cdc", starts, (ends - starts).astype(np.uint32))

    if want("gather"):
        # K8 peer gather on local memory (copy engine vs kernel; on the 8-GPU node the same launch
        # reads the peers' arenas over xGMI): 7 segments, as for 8 ranks
        seg = n // 8
        dst_g = ops.padded_empty(n, dev)
        srcs = [arena.data_ptr() + i * seg + 3 for i in range(7)]
        dsts = [dst_g.data_ptr() + i * seg + 3 for i in range(7)]
        ms = timed(lambda: H.peer_gather(srcs, dsts, [seg - 64] * 7, st), a.iters)
        emit(kernel="peer_gather_k8_local(7 segs)", bytes=7 * seg, ms=ms, gbps=7 * seg / ms / 1e6)
        assert torch.equal(dst_g[3:seg - 61], arena[3:seg - 61])

        def dma():
            for i in range(7):
                H.memcpy_async(dsts[i], srcs[i], seg - 64, st)
        ms = timed(dma, a.iters)
        emit(kernel="hipMemcpyAsync_local(7 segs)", bytes=7 * seg, ms=ms, gbps=7 * seg / ms / 1e6)
        del dst_g

    if want("cdc"):
        cap = n // 4096
        cand = torch.empty(cap, dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)

        def run_cdc():
            cnt.zero_()
            H.cdc_candidates(arena.data_ptr(), n, ops.XET_MASK, cand.data_ptr(), cnt.data_ptr(), cap, st)
        ms = timed(run_cdc, a.iters)
        emit(kernel="cdc_candidates", bytes=n, ms=ms, gbps=n / ms / 1e6, candidates=int(cnt.item()))

    # serialized xorb body of uncompressed chunks for place/index
    if want("place") or want("ingest"):
        body_n = nck * (csize + 8)
        body = ops.padded_empty(body_n, dev)
        data_off = offs
        out_off = np.arange(nck, dtype=np.uint64) * (csize + 8)
        ops.pack_chunks(arena, data_off, lens, out_off, body)
        dst = ops.padded_empty(n, dev)
        per_term = 1024  # 64 MiB terms
        nterm = (nck + per_term - 1) // per_term
        terms = np.zeros(nterm, dtype=ops.TERM_DTYPE)
        for t in range(nterm):
            c0, c1 = t * per_term, min(nck, (t + 1) * per_term)
            terms[t] = (c0 * (csize + 8), (c1 - c0) * (csize + 8), c0 * csize, c0, c1 - c0, (c1 - c0) * csize)
        ws = ops.IngestWorkspace(dev, nterm, nck)
        hashes = torch.empty((nck, 32), dtype=torch.uint8, device=dev)
        ms = timed(lambda: ops.ingest_terms(body, dst, terms, hashes, ws=ws, check=False), a.iters)
        emit(kernel="ingest_none(index+place+hash)", bytes=n, ms=ms, gbps=n / ms / 1e6)
        ops.raise_on_error(ws.err)
        assert torch.equal(dst[:1 << 20], arena[:1 << 20])
        tdev = ws.terms
        ms = timed(lambda: H.index_terms(body.data_ptr(), tdev.data_ptr(), nterm, ws.chunks.data_ptr(),
                                         ws.err.data_ptr(), st), a.iters)
        emit(kernel="index_terms", bytes=body_n, ms=ms, gbps=body_n / ms / 1e6, terms=nterm)
        ms = timed(lambda: H.place_chunks(body.data_ptr(), body_n, dst.data_ptr(), n, ws.chunks.data_ptr(), nck, 0,
                                          n, ws.err.data_ptr(), st), a.iters)
        emit(kernel="place_raw(+lz4 scan)", bytes=n, ms=ms, gbps=n / ms / 1e6)
        ms = timed(lambda: H.hash_chunks(dst.data_ptr(), n, ws.chunks.data_ptr(), nck, hashes.data_ptr(), 0, 0, st),
                   a.iters)
        emit(kernel="hash_chunks[wave]", bytes=n, ms=ms, gbps=n / ms / 1e6)
        sp, sb = hs.get(nck, n)
        ms = timed(lambda: H.hash_chunks(dst.data_ptr(), n, ws.chunks.data_ptr(), nck, hashes.data_ptr(), 0, 0, st,
                                         sp, sb), a.iters)
        emit(kernel="hash_chunks[flat]", bytes=n, ms=ms, gbps=n / ms / 1e6)
        del body, dst

    def ingest_case(name, raw, policy, iters, fused=None, after=None):
        """Pack `raw` into xorb runs with `policy`, then time index+place/decode+hash on the GPU
        (fused: one place+hash pass; None = the ZEST_FUSED_INGEST default).  `after(src, dst, ws,
        n_chunks)` runs extra timings on the indexed batch."""
        m = len(raw)
        ends = C.chunk_ends(raw)
        b = C.XorbBuilder(policy)
        prev, terms_l, bodies, src_off, cbase, schemes = 0, [], [], 0, 0, {}

        def close():
            nonlocal src_off, cbase
            body_b = b.serialize(False)
            for e in C.index_chunks(body_b):
                schemes[e[2]] = schemes.get(e[2], 0) + 1
            bodies.append(body_b)
            terms_l.append((src_off, len(body_b), cbase, b.num_chunks(), b.unpacked_size()))
            src_off += len(body_b)
            cbase += b.num_chunks()
            b.clear()

        for e in ends:
            if not b.fits(e - prev):
                close()
            b.add_chunk(raw[prev:e])
            prev = e
        close()
        blob = b"".join(bodies)
        terms = np.zeros(len(terms_l), dtype=ops.TERM_DTYPE)
        uo = 0
        for i, t in enumerate(terms_l):
            terms[i] = (t[0], t[1], uo, t[2], t[3], t[4])
            uo += t[4]
        src = ops.padded_empty(len(blob), dev)
        src.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
        dst = ops.padded_empty(m, dev)
        nck2 = int(terms["n_chunks"].sum())
        hashes = torch.empty((nck2, 32), dtype=torch.uint8, device=dev)
        ws = ops.IngestWorkspace(dev, len(terms), nck2)
        comp = policy != "none"
        ms = timed(lambda: ops.ingest_terms(src, dst, terms, hashes, ws=ws, check=False, fused=fused,
                                            has_compressed=comp), iters)
        ops.raise_on_error(ws.err)
        ok = dst[:m].cpu().numpy().tobytes() == raw
        tag = "" if fused is None else ("[fused]" if fused else "[place+hash]")
        emit(kernel=f"ingest_{policy}({name}){tag}", bytes=m, ms=ms, gbps=m / ms / 1e6, ratio=len(blob) / m,
             chunks=nck2, schemes={str(k): v for k, v in sorted(schemes.items())}, exact=ok)
        assert ok, name
        if after is not None:
            after(src, dst, ws, nck2)
        del src, dst, hashes, ws

    if want("lz4"):
        # bf16-like weights, compressed on the host (LZ4 / BG4 frames), decoded on the GPU
        m = min(n, 256 << 20)
        w = (np.random.default_rng(0).standard_normal(m // 2).astype(np.float32) * 0.02)
        raw = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
        for policy in ("lz4", "bg4"):
            ingest_case("bf16", raw, policy, a.iters)

    if want("lz4big"):
        # a bench-sized round: 1 GiB of bf16 weights = ~16.7k chunks
        m = 1 << 30
        w = (np.random.default_rng(0).standard_normal(m // 2).astype(np.float32) * 0.02)
        raw = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
        del w
        ingest_case("bf16_1g", raw, "bg4", max(3, a.iters // 4))
        del raw

    if want("lz4occ"):
        # K3 alone on a bench-sized BG4 round, persistent grid capped at 8 / 4 / 2 / 1 / 0.5 waves
        # per SIMD: latency-bound waves speed up with occupancy, an issue-bound decoder does not
        m = 1 << 30
        w = (np.random.default_rng(0).standard_normal(m // 2).astype(np.float32) * 0.02)
        raw = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
        del w

        def occ(src, dst, ws, n):
            for g in (2048, 1024, 512, 256, 128):
                ms = timed(lambda: H.lz4_decode(src.data_ptr(), src.numel(), dst.data_ptr(), dst.numel(),
                                                ws.chunks.data_ptr(), n, ws.err.data_ptr(), st, g), 3)
                ops.raise_on_error(ws.err)
                emit(kernel=f"lz4_decode(bf16_1g,grid={g})", bytes=m, ms=ms, gbps=m / ms / 1e6,
                     waves_per_simd=g * 4 / 1024)
            assert dst[:m].cpu().numpy().tobytes() == raw
            # the two-kernel decoder: lane-per-chunk parse into records, then record-driven execute
            dec = ops.DecodeScratch(dev)
            sp, sb = dec.get(n, src.numel())
            dst.zero_()
            ms = timed(lambda: H.lz4_decode(src.data_ptr(), src.numel(), dst.data_ptr(), dst.numel(),
                                            ws.chunks.data_ptr(), n, ws.err.data_ptr(), st, 0, sp, sb), 3)
            ops.raise_on_error(ws.err)
            fb = int((dec.buf[:4 * n].view(torch.int32) == -1).sum())
            emit(kernel="lz4_decode(bf16_1g,records)", bytes=m, ms=ms, gbps=m / ms / 1e6, scratch_mb=sb >> 20,
                 fallback_chunks=fb)
            assert dst[:m].cpu().numpy().tobytes() == raw

        ingest_case("bf16_1g", raw, "bg4", 3, after=occ)
        del raw

    if want("k3pair"):
        # round 4: producer/consumer wave pairs (k_lz4_pair) vs the one-wave decoder, and the serial
        # header walk k_index_terms, at a small launch (256 MiB, ~4 k chunks: fewer chunks than wave
        # slots) and a bench round (1 GiB).  (A scan-based header walk measured here at 5.4 / 12.3 ms
        # against 0.51 / 0.61 ms serial was removed: profiles/r4/kbench_k3pair_r4b.jsonl.)
        for m, tag in ((128 << 20, "bf16_128m"), (256 << 20, "bf16_256m"), (512 << 20, "bf16_512m"),
                       (768 << 20, "bf16_768m"), (1 << 30, "bf16_1g")):
            w = (np.random.default_rng(0).standard_normal(m // 2).astype(np.float32) * 0.02)
            raw = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
            del w

            def pair(src, dst, ws, n, m=m, tag=tag, raw=raw):
                for label, kw in (("one-wave", {}), ("pair", {"pair": True})):
                    dst.zero_()
                    ms = timed(lambda: H.lz4_decode(src.data_ptr(), src.numel(), dst.data_ptr(), dst.numel(),
                                                    ws.chunks.data_ptr(), n, ws.err.data_ptr(), st, 0, **kw), 5)
                    ops.raise_on_error(ws.err)
                    emit(kernel=f"lz4_decode({tag},{label})", bytes=m, ms=ms, gbps=m / ms / 1e6, chunks=n)
                    assert dst[:m].cpu().numpy().tobytes() == raw, label
                nt = ws.max_terms
                chunks0 = ws.chunks.clone()
                ws.err.zero_()
                ms = timed(lambda: H.index_terms(src.data_ptr(), ws.terms.data_ptr(), nt, ws.chunks.data_ptr(),
                                                 ws.err.data_ptr(), st), 5)
                ops.raise_on_error(ws.err)
                emit(kernel=f"index_terms({tag},serial)", bytes=src.numel(), ms=ms, gbps=src.numel() / ms / 1e6,
                     terms=nt, chunks=n, same_records=bool(torch.equal(ws.chunks, chunks0)))

            ingest_case(tag, raw, "bg4", 3, after=pair)
            del raw

    if want("fuse"):
        # a bench round of raw chunks (1 GiB random bytes): place then hash vs the fused one pass,
        # and the same for a BG4 bf16 round (decode + place/hash)
        m = 1 << 30
        raw = np.random.default_rng(2).integers(0, 256, m, dtype=np.uint8).tobytes()
        for fused in (False, True):
            ingest_case("random_1g", raw, "none", max(3, a.iters), fused=fused)
        w = (np.random.default_rng(0).standard_normal(m // 2).astype(np.float32) * 0.02)
        raw = (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
        del w
        for fused in (False, True):
            ingest_case("bf16_1g", raw, "bg4", max(3, a.iters // 4), fused=fused)
        del raw

    if want("lz4paths"):
        # one decoder path per data set: short matches, long literal runs, RLE, far matches
        m = 64 << 20
        rng = np.random.default_rng(1)
        sets = {
            "lowent": rng.integers(0, 8, m, dtype=np.uint8) * 31,
            "sparse": np.where(rng.random(m) < 0.02, rng.integers(0, 256, m), 0).astype(np.uint8),
            "mostly_random": np.where(rng.random(m) < 0.85, rng.integers(0, 256, m), 7).astype(np.uint8),
        }
        phrase = rng.integers(0, 256, 40_000, dtype=np.uint8)
        far = np.resize(phrase, m).copy()
        far[rng.integers(0, m, m // 64)] = rng.integers(0, 256, m // 64, dtype=np.uint8)
        sets["far_repeats"] = far
        for name, arr in sets.items():
            ingest_case(name, arr.tobytes(), "lz4", a.iters)

    if want("sha1"):
        # K6 parity row: sha1_info_hash over many xorb hashes at once (reference: 1 hash, 55 ns on a CPU core)
        nh = 1 << 22
        hs = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
        ms = timed(lambda: ops.sha1_info_hash(hs), a.iters)
        emit(kernel="sha1_info_hash_gpu", hashes=nh, ms=ms, ns_per_hash=ms * 1e6 / nh,
             mbps=nh * 44 / (ms / 1e3) / 2**20)
        del hs

    if want("blake3_64kb"):
        # parity row blake3_64kb_gpu: plain BLAKE3 of many 64 KiB buffers
        nb = 1 << 15
        offs = np.arange(nb, dtype=np.uint64) * 65536
        lens = np.full(nb, 65536, dtype=np.uint32)
        ms = timed(lambda: ops.hash_ranges(arena, offs, lens, key_mode=2), a.iters)
        emit(kernel="blake3_64kb_gpu", bytes=nb * 65536, ms=ms, mbps=nb * 65536 / (ms / 1e3) / 2**20)

    if want("merkle"):
        nl = 80_000
        hs = torch.randint(0, 256, (nl * 8, 32), dtype=torch.uint8, device=dev)
        sz = torch.randint(8192, 131072, (nl * 8,), dtype=torch.int64, device=dev)
        jobs = [(i * nl, nl) for i in range(8)]
        ms = timed(lambda: ops.merkle_roots(hs, sz, jobs), a.iters)
        emit(kernel="merkle_8x80k_leaves", ms=ms, leaves=nl * 8)

    if want("h2d"):
        pin = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
        d = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        ms = timed(lambda: d.copy_(pin, non_blocking=True), a.iters)
        emit(kernel="h2d_pinned_1GiB", bytes=1 << 30, ms=ms, gbps=(1 << 30) / ms / 1e6)


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(json.dumps({"total_s": time.time() - t0}))
