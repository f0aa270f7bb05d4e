"""Python GPU pull worker: pull a repository's Xet files with one GPU as decode/verify engine.

`zest pull <repo> --gpus N` runs the native worker (`zest_amd/_bin/zest-gpu-worker`,
csrc/gpurt/gpu_worker.cpp) when it is built; this module is the fallback and the library form.
Two launch shapes:

* independent (what the CLI does): one process per device, ZEST_GPU_RANK / ZEST_GPU_WORLD /
  ZEST_GPU_STATUS set, HIP_VISIBLE_DEVICES pinned; no process group -- files are independent, and
  each worker writes its own status JSON; the CLI fetches the regular files and writes the ref.
* torchrun (`python -m torch.distributed.run --nproc-per-node N -m zest_amd.multigpu ...`): ranks
  all-reduce their byte counts and rank 0 fetches the regular files and writes the ref.

Xet files are assigned by size (LPT); each worker fetches its files' compressed runs through the
native cache -> P2P -> CDN waterfall, decodes and verifies them on its GPU (`_hip.DeviceXetPull`)
and writes them into the HF-cache snapshot (file i's write overlaps file i + 1's pull).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from . import _core, ops
from .parallel import assign_owners, bind_local_numa, init_from_env


def cached_file_ok(repo: str, commit: str, f: dict, dst: str) -> bool:
    """A snapshot file counts as cached only when it is verified: a matching verified marker, or a
    re-hash that matches its Xet hash (then the marker is written).  Same rule as the host pull
    (csrc/core/pull.cpp); the reference trusts existence alone (main.zig:222-225)."""
    if not (os.path.exists(dst) and os.path.getsize(dst) == f["size"]):
        return False
    if _core.check_verified_marker(repo, commit, f["path"], f["xet_hash"], dst):
        return True
    if _core.xet_hash_of_file(dst) == f["xet_hash"]:
        _core.write_verified_marker(repo, commit, f["path"], f["xet_hash"], dst)
        return True
    return False


_PINNED: list = []


def write_device_file(buf: torch.Tensor, path: str, chunk: int = 256 << 20, slots: int = 3) -> None:
    """Write a device byte buffer to `path`: D2H of chunk k + 1 into pinned memory (side stream)
    overlaps the pwrite of chunk k (writer threads, GIL released), instead of one pageable `.cpu()`
    copy of the whole file followed by one single-threaded write."""
    from concurrent.futures import ThreadPoolExecutor

    n = buf.numel()
    if len(_PINNED) < slots or _PINNED[0].numel() < chunk:  # reused across files
        _PINNED[:] = [torch.empty(chunk, dtype=torch.uint8).pin_memory() for _ in range(slots)]
    stream = torch.cuda.Stream(buf.device)
    stream.wait_stream(torch.cuda.current_stream(buf.device))

    def put(ev, fd, host, m, off):
        ev.synchronize()
        view = memoryview(host.numpy())[:m]
        done = 0
        while done < m:
            done += os.pwrite(fd, view[done:], off + done)

    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        with ThreadPoolExecutor(slots) as ex:
            futs = [None] * slots
            for k, off in enumerate(range(0, n, chunk)):
                s = k % slots
                if futs[s] is not None:
                    futs[s].result()  # slot free: its previous chunk is on disk (page cache)
                m = min(chunk, n - off)
                with torch.cuda.stream(stream):
                    _PINNED[s][:m].copy_(buf[off:off + m], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                futs[s] = ex.submit(put, ev, fd, _PINNED[s], m, off)
            for f in futs:
                if f is not None:
                    f.result()
    finally:
        os.close(fd)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="zest pull --gpus N")
    ap.add_argument("repo")
    ap.add_argument("--revision", "-r", default="main")
    ap.add_argument("--peer", "-p", action="append", default=[])
    ap.add_argument("--tracker", "-t", default=None)
    ap.add_argument("--no-p2p", action="store_true")
    ap.add_argument("--no-dht", action="store_true")
    ap.add_argument("--dht-bootstrap", action="append", default=[])
    ap.add_argument("--repo-type", default="model")
    ap.add_argument("--include", action="append", default=[], help="only files ending in this suffix")
    ap.add_argument("--concurrency", "-j", type=int, default=16, help="fetch threads per GPU worker")
    ap.add_argument("--pipeline-depth", type=int, default=1024,
                    help="pinned staging ring per GPU worker, MB (network -> staging -> HBM)")
    # the reference ignores unknown flags (main.zig:98-119); so do the GPU workers
    a, _unknown = ap.parse_known_args(argv)
    independent = "ZEST_GPU_RANK" in os.environ and "RANK" not in os.environ
    if independent:  # one worker per device, started by the CLI; no process group
        rank, world = int(os.environ["ZEST_GPU_RANK"]), int(os.environ.get("ZEST_GPU_WORLD", "1"))
        dev = torch.device("cuda", 0)
    else:
        rank, world, local, dev = init_from_env()
    if independent or (world == 1 and "RANK" not in os.environ):
        torch.cuda.set_device(dev)
        bind_local_numa(dev)
    t0 = time.time()
    try:
        import psutil
        startup = t0 - psutil.Process().create_time()
    except Exception:  # noqa: BLE001 - diagnostics only
        startup = float("nan")
    commit, files = _core.list_repo_files(a.repo, a.revision, a.repo_type)
    commit = commit or a.revision
    if a.include:
        files = [f for f in files if any(f["path"].endswith(s) for s in a.include)]
    cfg = json.loads(_core.config_json())
    snap = os.path.join(cfg["hf_cache_dir"], _core.repo_folder_name(a.repo, a.repo_type), "snapshots", commit)
    xet = [f for f in files if f["xet_hash"]]
    regular = [f["path"] for f in files if not f["xet_hash"]]
    owners = assign_owners([f["size"] for f in xet], world)
    mine = [f for f, o in zip(xet, owners) if o == rank]
    if rank == 0:
        print(f"zest pull {a.repo} (revision: {a.revision}) on {world} GPU(s)", flush=True)
        print(f"Found {len(files)} files ({len(xet)} Xet-backed), snapshot {commit}", flush=True)
    p2p = not a.no_p2p
    done_bytes = 0
    failed = 0
    t_pull = t_write = 0.0
    if mine:
        dp = ops.hip().DeviceXetPull(a.repo, a.revision, a.repo_type, p2p, a.peer, a.tracker, not a.no_dht,
                                     a.dht_bootstrap, dev.index or 0, max(16, a.pipeline_depth) << 20, max(1, a.concurrency))
        todo = []
        for f in mine:
            dst = os.path.join(snap, f["path"])
            if cached_file_ok(a.repo, commit, f, dst):
                print(f"[rank {rank}] {f['path']} (cached)", flush=True)
                continue
            todo.append(f)
        bufs = [ops.padded_empty(f["size"], dev)[:f["size"]] for f in todo]
        torch.cuda.synchronize(dev)
        tp = time.time()

        def write_back(f, buf, s_):
            dst = os.path.join(snap, f["path"])
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            tmp = dst + ".incomplete"
            tw = time.time()
            if os.environ.get("ZEST_GPU_WRITER") == "simple":
                buf.cpu().numpy().tofile(tmp)
            else:
                write_device_file(buf, tmp)
            os.replace(tmp, dst)
            _core.write_verified_marker(a.repo, commit, f["path"], f["xet_hash"], dst)  # verified on the GPU
            print(f"[rank {rank}] {f['path']} [xet, gpu {dev.index}] {f['size'] / 1e6:.1f} MB "
                  f"verified ({s_['seconds']:.2f}s device pull)", flush=True)
            return time.time() - tw

        # File by file: the snapshot write of file i (writer thread: D2H + pwrite, GIL released)
        # overlaps the device pull of file i + 1 (the native pull releases the GIL too), and one
        # bad file does not sink the others.
        from concurrent.futures import ThreadPoolExecutor
        writes = []
        with ThreadPoolExecutor(1) as writer:
            for f, buf in zip(todo, bufs):
                try:
                    s_ = dp.pull_file(f["xet_hash"], buf.data_ptr(), f["size"])
                except Exception as e:  # noqa: BLE001 - counted as a failed file
                    print(f"[rank {rank}] {f['path']}: error {e}", file=sys.stderr, flush=True)
                    failed += 1
                    continue
                writes.append((f, writer.submit(write_back, f, buf, s_)))
            t_pull = time.time() - tp
            for f, fut in writes:
                try:
                    t_write += fut.result()
                    done_bytes += f["size"]
                except OSError as e:
                    print(f"[rank {rank}] {f['path']}: write failed: {e}", file=sys.stderr, flush=True)
                    failed += 1
        del bufs
        stats = json.loads(dp.stats_json())
    else:
        stats = {}
    if rank == 0 and regular and not independent:  # independent workers: the CLI fetches these
        r = _core.pull(a.repo, a.revision, p2p, a.peer, a.tracker, not a.no_dht, a.dht_bootstrap, regular, True, 0,
                       a.repo_type)
        failed += r["failed_files"]
    if independent:
        dt = time.time() - t0
        status = os.environ.get("ZEST_GPU_STATUS")
        if status:
            with open(status, "w") as fh:
                json.dump({"complete": True, "rank": rank, "world": world, "failed_files": failed, "bytes": done_bytes,
                           "seconds": round(dt, 3), "stats": stats}, fh)
        print(f"[gpu {rank}] {done_bytes / 1e9:.2f} GB in {dt:.1f}s (worker start {startup:.1f}s, device pulls "
              f"{t_pull:.1f}s, writes {t_write:.1f}s overlapped)", flush=True)
        return 1 if failed else 0
    if rank == 0:
        _core.write_ref(a.repo, a.revision, commit, a.repo_type)
    tot = torch.tensor([float(done_bytes), float(failed), float(stats.get("bytes_from_peer", 0)),
                        float(stats.get("bytes_from_cdn", 0)), float(stats.get("bytes_from_cache", 0))],
                       dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    dt = time.time() - t0
    status = os.environ.get("ZEST_GPU_STATUS")
    if rank == 0 and status:  # every rank reached the end: tells the CLI not to retry on fewer GPUs
        with open(status, "w") as fh:
            json.dump({"complete": True, "world": world, "failed_files": int(tot[1].item())}, fh)
    if rank == 0:
        b, f_, peer, cdn, cache = tot.tolist()
        src = peer + cdn + cache
        print(f"\nXorb fetch stats:\n  From peers:   {peer / 1e6:.1f} MB\n  From CDN:     {cdn / 1e6:.1f} MB\n"
              f"  From cache:   {cache / 1e6:.1f} MB\n  P2P ratio:    {100 * peer / src if src else 0:.1f}%", flush=True)
        print(f"\n{b / 1e9:.2f} GB verified on {world} GPU(s) in {dt:.1f}s ({b / dt / 1e9:.2f} GB/s; "
              f"rank 0: worker start {startup:.1f}s, device pulls {t_pull:.1f}s, snapshot writes {t_write:.1f}s "
              f"overlapped with them)",
              flush=True)
        print(f"\nDone! Model available at:\n  {snap}", flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 1 if int(tot[1].item()) else 0


if __name__ == "__main__":
    raise SystemExit(main())
