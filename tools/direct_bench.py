"""End-to-end device pull benchmark: `zest_amd.pull(repo, device="cuda:0", direct=True)` of a real
model layout from a peer, compared with the host path (`zest pull` to the HF cache, then GPU load
and verify).

The seeder is the HBM seeder (zest_amd.seed.HbmSeedServer): xorbs packed on the GPU, served over
BEP XET on loopback.  The fake Hub publishes metadata only (`add_world(payload=False)`), so every
Xet byte has to come from the peer; xorb GETs to the CDN would 404 and are counted.

    python tools/direct_bench.py [--model llama-3.1-8b] [--skip-host] [--out profiles/direct_8b.json]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import zest_amd  # noqa: E402
from zest_amd import device as zdev  # noqa: E402
from zest_amd import models, ops  # noqa: E402
from zest_amd.seed import HbmSeedServer, HbmXorbArena  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402
from zest_amd.testing import FakeHub  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3.1-8b")
    ap.add_argument("--mode", default="random", choices=["random", "bf16"],
                    help="bf16: N(0,0.02) bf16 weights stored as BG4-LZ4 frames, as Xet stores checkpoints "
                         "(the host path decodes them on the CPU, the GPU paths on the device)")
    ap.add_argument("--skip-host", action="store_true")
    ap.add_argument("--skip-gpu-cli", action="store_true")
    ap.add_argument("--skip-direct", action="store_true")
    ap.add_argument("--trace-host", default=None, help="ZEST_TRACE=<file.json> for the host zest pull")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--cli-configs", default="",
                    help="';'-separated env settings for repeated `zest pull --gpus 1` runs, e.g. "
                         "'ZEST_GPU_WRITERS=1;ZEST_GPU_WRITERS=2,ZEST_GPU_WRITE_SLOTS=3'")
    ap.add_argument("--host-after", action="store_true",
                    help="time the host pull again after the GPU CLI configs (order check)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    spec = models.get(a.model)
    t0 = time.time()
    world = SyntheticWorld(spec, seed=5, mode=a.mode, compression="bg4" if a.mode == "bf16" else "none")
    content = ops.padded_empty(world.arena_bytes, dev)
    world.generate_on_device(content)
    world.build_on_device(content)
    arena = HbmXorbArena(world, content)
    del content
    torch.cuda.empty_cache()
    srv = HbmSeedServer(arena)
    hub = FakeHub()
    hub.start()
    commit = hub.add_world(world, exact=True, payload=False)
    total = world.model_bytes
    print(f"[setup] {spec.repo_id}: {total / 1e9:.2f} GB, {world.n_chunks} chunks, {world.n_xorbs} xorbs in HBM "
          f"({time.time() - t0:.1f}s)", flush=True)
    work = Path(tempfile.mkdtemp(prefix="zest-direct-"))
    os.environ.update(hub.env(str(work / "direct")))  # separate caches: the host pull must not hit them
    peer = f"127.0.0.1:{srv.port}"
    res = {"model": a.model, "repo": spec.repo_id, "bytes": total, "chunks": world.n_chunks, "xorbs": world.n_xorbs,
           "source": "HBM seeder over BEP XET (loopback TCP)",
           "data": ("synthetic random-byte weights, real tensor shapes" if a.mode == "random" else
                    "synthetic N(0,0.02) bf16 weights, real tensor shapes, BG4-LZ4 frames (stored/raw "
                    f"{float(world.chunk_clen.sum()) / float(world.chunk_len.sum()):.3f})")}
    try:
        if not a.skip_direct:
            # warm-up on the smallest Xet file (connections, allocator, kernels)
            zest_amd._init()
            torch.cuda.synchronize()
            t0 = time.time()
            out = zest_amd.pull(spec.repo_id, device="cuda:0", direct=True, peers=[peer], dht=False, threads=a.threads)
            torch.cuda.synchronize()
            dt = time.time() - t0
            n = sum(v.numel() * v.element_size() for v in out.values())
            res.update(direct_s=round(dt, 3), direct_gbps=round(total / dt / 1e9, 3), tensors=len(out),
                       tensor_bytes=n, cdn_xorb_gets=hub.counters.get("xorb_missing", 0) + hub.counters.get("xorb_get", 0))
            print(f"[direct] network -> HBM, GPU decode + BLAKE3/Merkle verify: {total / dt / 1e9:.2f} GB/s "
                  f"({dt:.1f}s, {len(out)} tensors)", flush=True)
            del out
            torch.cuda.empty_cache()
            # same, without keeping the fetched runs in the disk xorb cache (pure network -> HBM)
            os.environ.update(hub.env(str(work / "direct_nocache")))
            os.environ["ZEST_CACHE_WRITES"] = "0"
            t0 = time.time()
            out = zest_amd.pull(spec.repo_id, device="cuda:0", direct=True, peers=[peer], dht=False, threads=a.threads)
            torch.cuda.synchronize()
            dt = time.time() - t0
            os.environ.pop("ZEST_CACHE_WRITES")
            res.update(direct_nocache_s=round(dt, 3), direct_nocache_gbps=round(total / dt / 1e9, 3))
            print(f"[direct, ZEST_CACHE_WRITES=0] {total / dt / 1e9:.2f} GB/s ({dt:.1f}s)", flush=True)
            del out
            torch.cuda.empty_cache()

        def settle():
            # every timed pull starts with no dirty page cache of an earlier one still being written
            t = time.time()
            os.sync()
            return round(time.time() - t, 3)

        def host_pull(tag):
            env = dict(os.environ, **hub.env(str(work / tag)))
            if a.trace_host:
                env["ZEST_TRACE"] = a.trace_host
            synced = settle()
            t0 = time.time()
            r = subprocess.run([str(ROOT / "zest_amd" / "_bin" / "zest"), "pull", spec.repo_id, "--peer", peer,
                                "--no-dht"], env=env, capture_output=True, text=True, timeout=3600)
            t1 = time.time()
            if r.returncode != 0:
                raise SystemExit(r.stdout[-2000:] + r.stderr[-2000:])
            return t0, t1, synced

        if not a.skip_host:
            t0, t1, synced = host_pull("host")
            snap = work / "host" / "hf" / "hub" / ("models--" + spec.repo_id.replace("/", "--")) / "snapshots" / commit
            hashes = {f.path: world.file_hash_hex(i) for i, f in enumerate(world.xet_files)}
            tensors = zdev.load_snapshot(str(snap), dev, hashes)
            torch.cuda.synchronize()
            t2 = time.time()
            res.update(host_pull_s=round(t1 - t0, 3), host_pull_gbps=round(total / (t1 - t0) / 1e9, 3),
                       load_verify_s=round(t2 - t1, 3), load_verify_gbps=round(total / (t2 - t1) / 1e9, 3),
                       host_path_gbps=round(total / (t2 - t0) / 1e9, 3), host_tensors=len(tensors),
                       host_presync_s=synced)
            print(f"[host] zest pull to disk {total / (t1 - t0) / 1e9:.2f} GB/s, then load + GPU verify "
                  f"{total / (t2 - t1) / 1e9:.2f} GB/s -> end to end {total / (t2 - t0) / 1e9:.2f} GB/s", flush=True)
            del tensors
            subprocess.run(["rm", "-rf", str(work / "host")])
        if not a.skip_gpu_cli:
            # `zest pull --gpus 1`: the CLI's GPU worker (native zest-gpu-worker) pulls device-direct,
            # decodes + verifies on the GPU and writes the HF-cache snapshot
            configs = [c for c in a.cli_configs.split(";")] if a.cli_configs else [""]
            for ci, cfg in enumerate(configs):
                extra = dict(kv.split("=", 1) for kv in cfg.split(",") if kv)
                env = dict(os.environ, **hub.env(str(work / f"gpucli{ci}")), **extra)
                synced = settle()
                t0 = time.time()
                r = subprocess.run([str(ROOT / "zest_amd" / "_bin" / "zest"), "pull", spec.repo_id, "--peer", peer,
                                    "--no-dht", "--gpus", "1"], env=env, capture_output=True, text=True, timeout=3600)
                dt = time.time() - t0
                if r.returncode != 0:
                    raise SystemExit(r.stdout[-2000:] + r.stderr[-2000:])
                tail = [ln for ln in r.stdout.splitlines() if "verified on" in ln]
                workers = [ln for ln in r.stdout.splitlines() if ln.startswith("[gpu") and (" GB in " in ln or "timeline" in ln)]
                key = "gpu_cli" if not cfg else f"gpu_cli[{cfg}]"
                res[key] = {"s": round(dt, 3), "gbps": round(total / dt / 1e9, 3), "workers": workers, "presync_s": synced}
                if not cfg:
                    res.update(gpu_cli_pull_s=round(dt, 3), gpu_cli_pull_gbps=round(total / dt / 1e9, 3),
                               gpu_cli_summary=tail[-1] if tail else "", gpu_cli_workers=workers)
                for ln in workers + tail[-1:]:
                    print(f"[gpu cli worker {cfg}] {ln}", flush=True)
                print(f"[gpu cli {cfg}] zest pull --gpus 1 to disk: {total / dt / 1e9:.2f} GB/s ({dt:.1f}s)", flush=True)
                subprocess.run(["rm", "-rf", str(work / f"gpucli{ci}")])
        if a.host_after:
            t0, t1, synced = host_pull("host_after")
            res.update(host_after_s=round(t1 - t0, 3), host_after_gbps=round(total / (t1 - t0) / 1e9, 3))
            print(f"[host, again] zest pull to disk {total / (t1 - t0) / 1e9:.2f} GB/s", flush=True)
            subprocess.run(["rm", "-rf", str(work / "host_after")])
        res["seeder"] = srv.stats()
        print(json.dumps(res), flush=True)
        if a.out:
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
        return 0
    finally:
        srv.stop()
        hub.stop()
        subprocess.run(["rm", "-rf", str(work)])


if __name__ == "__main__":
    raise SystemExit(main())
