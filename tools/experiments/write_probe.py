"""How fast can one process put 16 GB of snapshot files on this machine's disk?  (host only, no GPU)

The GPU CLI pull (`zest pull --gpus 1`) verifies a model in HBM in ~1 s; what is left is writing the
snapshot files.  This probe times the candidate write strategies on 4 files x `--gb/4` GB, from a
256 MiB page-aligned source buffer (what the worker's pinned D2H slot is), each case starting after
`sync` with no dirty pages of an earlier case around:

  seq1      1 thread, files one after another, 256 MiB pwrite calls
  file4     4 threads, one file each
  split16   16 threads, 4 per file, disjoint ranges of a pre-sized file (pwrite)
  mmap16    16 threads, 4 per file, memcpy into a MAP_SHARED mapping of a pre-sized file
  direct4   O_DIRECT, 4 threads one file each
  direct16  O_DIRECT, 16 threads 4 per file, fallocate'd file
  one1/one4 ONE file (gb/4) written by 1 / 4 threads (does the inode lock serialize writers?)

`write_s` is the time until the last write call returned (what a pull waits for); `sync_s` the
time the following `sync` took (writeback the kernel still owed).

    python tools/experiments/write_probe.py [--gb 16] [--dir DIR] [--cases seq1,file4,...]
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import shutil
import tempfile
import threading
import time

import numpy as np

PIECE = 256 << 20


def _src() -> memoryview:
    m = mmap.mmap(-1, PIECE)  # page aligned: usable for O_DIRECT
    a = np.frombuffer(m, dtype=np.uint8)
    a[:] = np.random.default_rng(0).integers(0, 256, PIECE, dtype=np.uint8)
    return memoryview(m)


def _ranges(size: int, parts: int):
    step = -(-size // parts)
    step = -(-step // PIECE) * PIECE
    return [(o, min(size, o + step)) for o in range(0, size, step)]


def _pwrite_range(fd: int, src: memoryview, lo: int, hi: int) -> None:
    off = lo
    while off < hi:
        n = min(PIECE, hi - off)
        done = 0
        while done < n:
            done += os.pwrite(fd, src[done:n], off + done)
        off += n


def _mmap_range(mm: mmap.mmap, src: memoryview, lo: int, hi: int) -> None:
    dst = np.frombuffer(mm, dtype=np.uint8)
    s = np.frombuffer(src, dtype=np.uint8)
    off = lo
    while off < hi:
        n = min(PIECE, hi - off)
        np.copyto(dst[off:off + n], s[:n])
        off += n


def run_case(case: str, d: str, size: int, src: memoryview) -> dict:
    if case in ("one1", "one4"):  # ONE file: does a second writer help (inode lock)?
        p = os.path.join(d, "one.bin")
        fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        os.ftruncate(fd, size)
        parts = _ranges(size, 1 if case == "one1" else 4)
        t0 = time.perf_counter()
        th = [threading.Thread(target=_pwrite_range, args=(fd, src, lo, hi)) for lo, hi in parts]
        for t in th:
            t.start()
        for t in th:
            t.join()
        t1 = time.perf_counter()
        os.close(fd)
        os.sync()
        t2 = time.perf_counter()
        os.unlink(p)
        return {"case": case, "threads": len(parts), "GB": round(size / 1e9, 2), "write_s": round(t1 - t0, 3),
                "GBps": round(size / (t1 - t0) / 1e9, 2), "sync_s": round(t2 - t1, 3)}
    paths = [os.path.join(d, f"f{i}.bin") for i in range(4)]
    jobs = []  # (callable)
    fds, maps = [], []
    direct = case.startswith("direct")
    flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC | (os.O_DIRECT if direct else 0)
    if case in ("split16", "mmap16", "direct16"):
        for p in paths:
            fd = os.open(p, (os.O_RDWR | os.O_CREAT | os.O_TRUNC) if case == "mmap16" else flags, 0o644)
            if case == "direct16":
                os.posix_fallocate(fd, 0, size)
            else:
                os.ftruncate(fd, size)
            fds.append(fd)
            if case == "mmap16":
                mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_WRITE | mmap.PROT_READ)
                maps.append(mm)
                jobs += [lambda mm=mm, lo=lo, hi=hi: _mmap_range(mm, src, lo, hi) for lo, hi in _ranges(size, 4)]
            else:
                jobs += [lambda fd=fd, lo=lo, hi=hi: _pwrite_range(fd, src, lo, hi) for lo, hi in _ranges(size, 4)]
    else:
        for p in paths:
            fds.append(os.open(p, flags, 0o644))
        if case == "seq1":
            jobs = [lambda: [_pwrite_range(fd, src, 0, size) for fd in fds]]
        else:
            jobs = [lambda fd=fd: _pwrite_range(fd, src, 0, size) for fd in fds]
    errs = []

    def wrap(j):
        try:
            j()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    t0 = time.perf_counter()
    th = [threading.Thread(target=wrap, args=(j,)) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    t1 = time.perf_counter()
    for mm in maps:
        mm.close()
    for fd in fds:
        os.close(fd)
    t2 = time.perf_counter()
    os.sync()
    t3 = time.perf_counter()
    for p in paths:
        os.unlink(p)
    total = 4 * size
    return {"case": case, "threads": len(jobs), "GB": round(total / 1e9, 2), "write_s": round(t1 - t0, 3),
            "GBps": round(total / (t1 - t0) / 1e9, 2), "close_s": round(t2 - t1, 3), "sync_s": round(t3 - t2, 3),
            "errors": errs[:2]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=16.0)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--cases", default="seq1,file4,split16,mmap16,direct4,direct16")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="zest-wprobe-", dir=a.dir)
    size = int(a.gb * 1e9 / 4) // PIECE * PIECE
    src = _src()
    rows = []
    try:
        st = os.statvfs(d)
        print(f"[dir] {d} free {st.f_bavail * st.f_frsize / 1e9:.0f} GB", flush=True)
        os.sync()
        for c in a.cases.split(","):
            r = run_case(c, d, size, src)
            rows.append(r)
            print(json.dumps(r), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(json.dumps(r) for r in rows) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
