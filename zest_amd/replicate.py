"""One command, every tensor on every GPU of the node:

    python -m zest_amd pull meta-llama/Llama-3.1-70B --gpus 8 --device all [--save-snapshot]
    zest pull meta-llama/Llama-3.1-70B --gpus 8 --device all          (the `zest` console script)

The launcher (this process) makes no GPU call: it starts N rank processes -- RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_* set, one per GPU, as torchrun would -- and waits for them.  Each rank joins the
process group (RCCL when every rank has its own GPU; gloo with the ranks sharing the devices
otherwise, or with --backend gloo) and runs the intra-node swarm pull
(zest_amd.parallel.swarm_pull = zest_amd.pull(device="all")): every rank fetches a byte-balanced
share of the model's terms device-direct, the shares are replicated over xGMI, every rank verifies
its whole replica.  With --save-snapshot rank 0 also writes the verified files into the HF-cache
snapshot (plus the repository's non-safetensors files and the ref), so `from_pretrained` works from
disk afterwards.  Every rank writes a status JSON; the launcher prints one status line per rank and
returns non-zero if any rank failed.

A library user who already runs under torchrun calls zest_amd.pull(repo, device="all") instead.
Reference: the reference's whole UX is one command (src/main.zig:83-305); it has no multi-GPU
placement at all.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time


def parse_args(argv):
    ap = argparse.ArgumentParser(prog="zest pull --device all")
    ap.add_argument("repo")
    ap.add_argument("--revision", "-r", default="main")
    ap.add_argument("--gpus", type=int, default=0, help="ranks (default: every visible GPU, else 1)")
    ap.add_argument("--device", default="all", choices=["all"])
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="auto: RCCL when every rank has a GPU of its own, else gloo (ranks share devices)")
    ap.add_argument("--cpu", action="store_true", help="host memory instead of GPUs (gloo; tests)")
    ap.add_argument("--save-snapshot", action="store_true", help="rank 0 writes the HF-cache snapshot too")
    ap.add_argument("--peer", "-p", action="append", default=[])
    ap.add_argument("--tracker", "-t", default=None)
    ap.add_argument("--no-p2p", action="store_true")
    ap.add_argument("--no-dht", action="store_true")
    ap.add_argument("--dht-bootstrap", action="append", default=[])
    ap.add_argument("--repo-type", default="model")
    ap.add_argument("--exchange", default="auto")
    ap.add_argument("--round-mb", type=int, default=0)
    ap.add_argument("--concurrency", "-j", type=int, default=16, help="fetch threads per rank")
    ap.add_argument("--timeout", type=float, default=0, help="launcher: kill the ranks after this many seconds")
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    a, _unknown = ap.parse_known_args(argv)  # (the reference ignores unknown flags, main.zig:98-119)
    return a


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_gpus() -> int:
    # counting devices does not initialise the GPU on this image (no HIP context is created)
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def launch(argv) -> int:
    """Start the ranks (before anything here touches a GPU) and wait for them."""
    a = parse_args(argv)
    n = a.gpus or (1 if a.cpu else max(1, _visible_gpus()))
    port = str(_free_port())
    status_dir = tempfile.mkdtemp(prefix="zest-replicate-")
    procs = []
    t0 = time.time()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   ZEST_REPLICATE_STATUS=os.path.join(status_dir, f"rank{r}.json"))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        cmd = [sys.executable, "-m", "zest_amd.replicate", "--worker", *argv]
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    print(f"zest pull {a.repo} (revision: {a.revision}) onto {n} rank(s), every tensor on every rank", flush=True)
    codes = [None] * n
    deadline = t0 + a.timeout if a.timeout > 0 else None
    failed_at = None
    try:
        while any(c is None for c in codes):
            for i, p in enumerate(procs):
                if codes[i] is None:
                    codes[i] = p.poll()
                    if codes[i] not in (None, 0) and failed_at is None:
                        failed_at = time.time()
            now = time.time()
            # a failed rank: the others get a grace period (the swarm's own recovery may finish
            # without it), then the whole job is torn down rather than left waiting on a peer
            if (failed_at is not None and now - failed_at > 60) or (deadline is not None and now > deadline):
                for i, p in enumerate(procs):
                    if codes[i] is None:
                        try:
                            os.killpg(p.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
                for i, p in enumerate(procs):
                    if codes[i] is None:
                        try:
                            codes[i] = p.wait(timeout=10)
                        except subprocess.TimeoutExpired:
                            os.killpg(p.pid, signal.SIGKILL)
                            codes[i] = p.wait()
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        return 130
    stats = []
    for r in range(n):
        try:
            with open(os.path.join(status_dir, f"rank{r}.json")) as fh:
                stats.append(json.load(fh))
        except (OSError, ValueError):
            stats.append(None)
    for r, (c, st) in enumerate(zip(codes, stats)):
        if st and st.get("ok"):
            print(f"[rank {r}] {st['device']}: {st['tensors']} tensors, {st['bytes'] / 1e9:.2f} GB verified in "
                  f"{st['seconds']:.2f}s; fetched {st['fetched_bytes'] / 1e9:.2f} GB, received "
                  f"{st['received_bytes'] / 1e9:.2f} GB from peers (exchange {st['exchange']})", flush=True)
        else:
            print(f"[rank {r}] FAILED (exit {c}): {(st or {}).get('error', 'no status')}", flush=True)
    ok = all(c == 0 for c in codes) and all(st and st.get("ok") for st in stats)
    if ok:
        total = stats[0]["bytes"]
        wall = time.time() - t0
        print(f"\n{total / 1e9:.2f} GB resident and verified on each of {n} rank(s) in {wall:.1f}s "
              f"({n * total / wall / 1e9:.2f} GB/s aggregate)", flush=True)
        if stats[0].get("snapshot"):
            print(f"\nDone! Model available at:\n  {stats[0]['snapshot']}", flush=True)
    return 0 if ok else 1


def worker(a) -> int:
    import torch
    import torch.distributed as dist

    from . import _core
    from .parallel import bind_local_numa, swarm_pull

    rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
    status = os.environ.get("ZEST_REPLICATE_STATUS")
    rec = {"rank": rank, "world": world, "ok": False}
    t0 = time.time()
    try:
        n_dev = 0 if a.cpu else torch.cuda.device_count()
        if n_dev:
            dev = torch.device("cuda", local % n_dev)
            torch.cuda.set_device(dev)
            bind_local_numa(dev)
        else:
            dev = torch.device("cpu")
        backend = a.backend
        if backend == "auto":
            backend = "nccl" if n_dev >= world else "gloo"
        import datetime
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600), **kw)
        rec["device"], rec["backend"] = str(dev), backend
        st: dict = {}
        files: dict = {}
        out = swarm_pull(a.repo, a.revision, device=dev, p2p=not a.no_p2p, peers=a.peer, tracker=a.tracker,
                         dht=not a.no_dht, dht_bootstrap=a.dht_bootstrap, repo_type=a.repo_type,
                         threads=max(1, a.concurrency), exchange=a.exchange, stats=st,
                         round_bytes=(a.round_mb << 20) if a.round_mb else None,
                         files_out=files if (a.save_snapshot and rank == 0) else None)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        rec.update(tensors=len(out), bytes=int(st.get("total_bytes", 0)), seconds=round(time.time() - t0, 3),
                   fetched_bytes=int(st.get("fetched_bytes", 0)), received_bytes=int(st.get("received_bytes", 0)),
                   exchange=st.get("exchange"), p2p_ratio=st.get("p2p_ratio"), phases=st.get("phases"))
        if a.save_snapshot and rank == 0:
            rec["snapshot"] = _write_snapshot(a, files)
        del out, files
        rec["ok"] = True
    except Exception as e:  # noqa: BLE001 - reported through the status file
        rec["error"] = f"{type(e).__name__}: {e}"[:2000]
        print(f"[rank {rank}] {rec['error']}", file=sys.stderr, flush=True)
    finally:
        if status:
            with open(status + ".tmp", "w") as fh:
                json.dump(rec, fh)
            os.replace(status + ".tmp", status)
    try:
        if dist.is_initialized():
            if rec["ok"]:
                dist.barrier()
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass
    return 0 if rec["ok"] else 1


def _write_snapshot(a, files: dict) -> str:
    """Rank 0: the verified files into the HF-cache snapshot (device buffers through the pipelined
    pinned writer), the repository's other files through the host pull, then the ref."""
    import torch

    from . import _core
    commit, listing = _core.list_repo_files(a.repo, a.revision, a.repo_type)
    commit = commit or a.revision
    cfg = json.loads(_core.config_json())
    snap = os.path.join(cfg["hf_cache_dir"], _core.repo_folder_name(a.repo, a.repo_type), "snapshots", commit)
    by_path = {f["path"]: f for f in listing}
    for path, buf in files.items():
        dst = os.path.join(snap, path)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        tmp = dst + ".incomplete"
        if buf.device.type == "cuda":
            from .multigpu import write_device_file
            write_device_file(buf, tmp)
        else:
            buf.numpy().tofile(tmp)
        os.replace(tmp, dst)
        f = by_path.get(path)
        if f and f.get("xet_hash"):
            _core.write_verified_marker(a.repo, commit, path, f["xet_hash"], dst)  # verified on the device
    rest = [f["path"] for f in listing if f["path"] not in files]
    if rest:
        r = _core.pull(a.repo, a.revision, not a.no_p2p, a.peer, a.tracker, not a.no_dht, a.dht_bootstrap, rest,
                       True, 0, a.repo_type)
        if r["failed_files"]:
            raise RuntimeError(f"{r['failed_files']} non-safetensors file(s) failed")
    _core.write_ref(a.repo, a.revision, commit, a.repo_type)
    del torch
    return snap


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    if a.worker:
        return worker(a)
    return launch([x for x in argv if x != "--worker"])


if __name__ == "__main__":
    sys.exit(main())
