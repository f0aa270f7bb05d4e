"""`zest bench --gpu`: the device rows of the benchmark harness, in the reference's JSON schema.

The reference's `zest bench --synthetic` (src/bench.zig:150-287) times five host loops and prints
`{"results": [{name, runs, median_ns, throughput_mbps, bytes_processed}]}` (throughput in MiB/s,
bench.zig:28-33).  These rows time the MI355X kernels of the same pipeline with HIP events, one
row per kernel, in that schema (median over `runs` launches; throughput = bytes / 2^20 / s):

  blake3_64kb_gpu      keyed BLAKE3 of many 64 KiB chunks (K1; the reference's blake3_64kb row)
  blake3_cdc_gpu       the same over Xet CDC chunks (8-128 KiB), as a pull hashes them
  sha1_info_hash_gpu   SHA-1 info-hashes of 44-byte messages (K6; the reference's sha1_info_hash)
  cdc_gpu              GearHash CDC boundary candidates (K5)
  xorb_verify_gpu      header walk + placement + BLAKE3 of uncompressed xorb runs (K4 fused ingest)
  lz4_decode_gpu       the same for BG4-LZ4 bf16 weights (K3 batched decoder + K1)
  lz4_decode_gpu_hostidx  the same batch the way the public device path (DeviceXetPull) runs it:
                       chunk records come from the header index the fetch workers build while
                       validating each run (host, outside the timed region), so the device work is
                       the records' H2D upload + decode + fused place/hash -- no device header walk
  merkle_gpu           Xet Merkle file hashes over 8 x 80k leaves (K2)
  h2d_pinned_gpu       pinned host -> HBM copy (the ingest ceiling of a one-GPU pull)
  rccl_allgather_xorb  (N ranks) RCCL all-gather of 64 MiB xorb slabs over xGMI, bytes received
                       per GPU (the piece exchange of the intra-node swarm)

    python -m zest_amd.gpubench [--json] [--mib 1024] [--runs 5]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m zest_amd.gpubench --json   # + RCCL row
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

from . import _core, ops


def _time(fn, runs: int) -> float:
    """Median ns of `runs` launches of fn (after one warm-up), HIP events."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(runs):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e6)
    return float(np.median(ts))


def _row(name: str, runs: int, median_ns: float, nbytes: int) -> dict:
    return {"name": name, "runs": runs, "median_ns": int(median_ns),
            "throughput_mbps": round(nbytes / 2**20 / (median_ns / 1e9), 2) if median_ns > 0 else 0.0,
            "bytes_processed": int(nbytes)}


def _xorb_runs(raw: bytes, policy: str):
    """Serialized xorb runs (host XorbBuilder) of `raw` + the TERM_DTYPE records that ingest them."""
    ends = _core.chunk_ends(raw)
    b = _core.XorbBuilder(policy)
    bodies, terms_l, src_off, cbase, prev = [], [], 0, 0, 0

    def close():
        nonlocal src_off, cbase
        body = b.serialize(False)
        bodies.append(body)
        terms_l.append((src_off, len(body), cbase, b.num_chunks(), b.unpacked_size()))
        src_off += len(body)
        cbase += b.num_chunks()
        b.clear()

    for e in ends:
        if not b.fits(e - prev):
            close()
        b.add_chunk(raw[prev:e])
        prev = e
    close()
    terms = np.zeros(len(terms_l), dtype=ops.TERM_DTYPE)
    uo = 0
    for i, t in enumerate(terms_l):
        terms[i] = (t[0], t[1], uo, t[2], t[3], t[4])
        uo += t[4]
    return b"".join(bodies), terms, cbase


def run(mib: int = 1024, runs: int = 5, device="cuda:0") -> list[dict]:
    dev = torch.device(device)
    torch.cuda.set_device(dev)
    H = ops.hip()
    st = torch.cuda.current_stream(dev).cuda_stream
    rows = []
    n = mib << 20
    arena = ops.padded_empty(n, dev)
    ops.fill_synthetic(arena, 1, 0, 0)

    nb = n // 65536
    offs = torch.from_numpy((np.arange(nb, dtype=np.uint64) * 65536).view(np.int64)).to(dev)
    lens = torch.full((nb,), 65536, dtype=torch.int32, device=dev)
    out = torch.empty((nb, 32), dtype=torch.uint8, device=dev)
    hs = ops.HashScratch(dev)
    sp, sb = hs.get(nb, nb * 65536)
    ns = _time(lambda: H.hash_ranges(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(), nb, out.data_ptr(),
                                     ops.KEY_DATA, st, sp, sb), runs)
    rows.append(_row("blake3_64kb_gpu", runs, ns, nb * 65536))
    # the same bytes cut like a real pull: Xet CDC chunks (8-128 KiB)
    ends = _core.chunk_ends(arena[: min(n, 256 << 20)].cpu().numpy().tobytes())
    cst = np.concatenate([[0], np.asarray(ends[:-1], dtype=np.int64)])
    clen = np.diff(np.concatenate([[0], np.asarray(ends, dtype=np.int64)]))
    coffs = torch.from_numpy(cst).to(dev)
    clens = torch.from_numpy(clen.astype(np.int32)).to(dev)
    cout = torch.empty((len(ends), 32), dtype=torch.uint8, device=dev)
    sp, sb = hs.get(len(ends), int(clen.sum()))
    ns = _time(lambda: H.hash_ranges(arena.data_ptr(), coffs.data_ptr(), clens.data_ptr(), len(ends), cout.data_ptr(),
                                     ops.KEY_DATA, st, sp, sb), runs)
    rows.append(_row("blake3_cdc_gpu", runs, ns, int(clen.sum())))

    nh = 1 << 22
    hs = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
    ns = _time(lambda: ops.sha1_info_hash(hs), runs)
    rows.append(_row("sha1_info_hash_gpu", runs, ns, nh * 44))
    del hs

    cap = n // 4096
    cand = torch.empty(cap, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)

    def cdc():
        cnt.zero_()
        H.cdc_candidates(arena.data_ptr(), n, ops.XET_MASK, cand.data_ptr(), cnt.data_ptr(), cap, st)
    rows.append(_row("cdc_gpu", runs, _time(cdc, runs), n))
    del cand

    m = min(n, 256 << 20)  # host-built xorbs: keep the host packing time bounded
    for name, raw, policy in (("xorb_verify_gpu", arena[:m].cpu().numpy().tobytes(), "none"),
                              ("lz4_decode_gpu", _bf16(m), "bg4")):
        blob, terms, nck = _xorb_runs(raw, policy)
        src = ops.padded_empty(len(blob), dev)
        src.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
        dst = ops.padded_empty(len(raw), dev)
        hashes = torch.empty((nck, 32), dtype=torch.uint8, device=dev)
        ws = ops.IngestWorkspace(dev, len(terms), nck)
        comp = policy != "none"
        ns = _time(lambda: ops.ingest_terms(src, dst, terms, hashes, ws=ws, check=False, has_compressed=comp), runs)
        ops.raise_on_error(ws.err)
        if dst[:len(raw)].cpu().numpy().tobytes() != raw:
            raise RuntimeError(f"{name}: decoded bytes differ from the input")
        rows.append(_row(name, runs, ns, len(raw)))
        if comp:
            rows.append(_hostidx_row(H, st, blob, raw, terms, nck, src, dst, hashes, ws, runs))
        del src, dst, hashes, ws

    nl = 80_000
    lh = torch.randint(0, 256, (nl * 8, 32), dtype=torch.uint8, device=dev)
    sz = torch.randint(8192, 131072, (nl * 8,), dtype=torch.int64, device=dev)
    jobs = [(i * nl, nl) for i in range(8)]
    rows.append(_row("merkle_gpu", runs, _time(lambda: ops.merkle_roots(lh, sz, jobs), runs), nl * 8 * 32))
    del lh, sz

    pin = torch.empty(min(n, 1 << 30), dtype=torch.uint8).pin_memory()
    d = torch.empty(pin.numel(), dtype=torch.uint8, device=dev)
    rows.append(_row("h2d_pinned_gpu", runs, _time(lambda: d.copy_(pin, non_blocking=True), runs), pin.numel()))
    del pin, d

    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        world = dist.get_world_size()
        slab = 64 << 20
        mine = torch.empty(slab, dtype=torch.uint8, device=dev)
        every = torch.empty(world * slab, dtype=torch.uint8, device=dev)
        dist.barrier()
        ns = _time(lambda: dist.all_gather_into_tensor(every, mine), runs)
        t = torch.tensor([ns], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rows.append(_row("rccl_allgather_xorb", runs, float(t.item()), (world - 1) * slab))
    return rows


def _hostidx_row(H, st, blob, raw, terms, nck, src, dst, hashes, ws, runs) -> dict:
    """lz4_decode_gpu_hostidx: records from the host header walk (_core.index_runs over the runs in
    pinned memory, as DeviceXetPull's fetch workers produce them), then per launch: records H2D +
    fused decode/place/hash.  Checked byte-exact and hash-equal to the device-walk row."""
    want = hashes.clone()
    pin = torch.frombuffer(bytearray(blob), dtype=torch.uint8).pin_memory()
    nrec = nck * ops.CHUNK_DTYPE.itemsize
    rec = torch.empty(nrec, dtype=torch.uint8).pin_memory()
    th = np.ascontiguousarray(terms, dtype=ops.TERM_DTYPE)
    e = _core.index_runs(pin.data_ptr(), len(blob), th.ctypes.data, len(th), rec.data_ptr(), nck)
    if e:
        raise RuntimeError(f"lz4_decode_gpu_hostidx: host header walk failed ({e:#x})")
    sp, sb = ws.hash_scratch.get(nck, len(raw))

    def launch():
        H.memcpy_async(ws.chunks.data_ptr(), rec.data_ptr(), nrec, st)
        H.ingest_chunks(src.data_ptr(), len(blob), dst.data_ptr(), dst.numel(), ws.chunks.data_ptr(), nck, True,
                        ws.err.data_ptr(), hashes.data_ptr(), 0, 0, st, sp, sb)
    dst.zero_()
    hashes.zero_()
    ws.err.zero_()
    ns = _time(launch, runs)
    ops.raise_on_error(ws.err)
    if dst[:len(raw)].cpu().numpy().tobytes() != raw or not torch.equal(hashes, want):
        raise RuntimeError("lz4_decode_gpu_hostidx: result differs from the device-walk ingest")
    return _row("lz4_decode_gpu_hostidx", runs, ns, len(raw))


def _bf16(nbytes: int) -> bytes:
    w = np.random.default_rng(0).standard_normal(nbytes // 2).astype(np.float32) * 0.02
    return (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="zest bench --gpu")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--mib", type=int, default=int(os.environ.get("ZEST_GPUBENCH_MIB", "1024")),
                    help="buffer size per row (env ZEST_GPUBENCH_MIB)")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args(argv)
    if not torch.cuda.is_available():
        print("zest bench --gpu: no GPU visible", file=sys.stderr)
        return 2
    t0 = time.time()
    rank = 0
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # torchrun: one rank per GPU, RCCL row added
        from .parallel import init_from_env
        rank, _world, _local, dev = init_from_env()
        a.device = str(dev)
    rows = run(a.mib, a.runs, a.device)
    if rank != 0:
        return 0
    if a.json:
        print(json.dumps({"results": rows, "device": torch.cuda.get_device_name(0)}))
    else:
        print(f"\nzest GPU benchmark results ({torch.cuda.get_device_name(0)}, {time.time() - t0:.1f}s)")
        print(f"{'Benchmark':<22}{'Runs':>8}{'Median (ns)':>16}{'MB/s':>14}")
        for r in rows:
            print(f"{r['name']:<22}{r['runs']:>8}{r['median_ns']:>16}{r['throughput_mbps']:>14.1f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
