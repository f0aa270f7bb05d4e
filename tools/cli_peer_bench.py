#!/usr/bin/env python3
"""`zest pull --gpus 1` vs the host `zest pull`, both from warm `zest serve` seeders (the native
BEP XET server reading its xorb cache through the page cache -- a source that is not itself the
bound, unlike the one HbmSeedServer process of tools/direct_bench.py).

A repo of bf16 weights (N(0, 0.02), BG4-LZ4 frames as Xet stores bf16 checkpoints) or random bytes
is published on the fake Hub; seeder 0 pulls it from the CDN, the other seeders copy its xorb cache,
all run `zest serve`.  Then, with `sync` before each timed run:
  host   `zest pull --peer ...`            CPU LZ4/BG4 decode + BLAKE3, file write, cache copy
  gpu    `zest pull --peer ... --gpus 1`   the native GPU worker: device decode + BLAKE3/Merkle,
                                           write-back from HBM, write-behind cache copy
  host, gpu again (order check; best of two each), after one untimed warm-up pull
Every pull verifies every file hash; snapshots are checked byte for byte.

    python tools/cli_peer_bench.py [--mb 4096] [--shards 4] [--mode bf16|random] [--seeders 1] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from e2e_util import Node, assert_snapshot, p2p_ratio  # noqa: E402
from zest_amd.testing import FakeHub  # noqa: E402


def weights(mode: str, nbytes: int, seed: int) -> bytes:
    rng = np.random.default_rng(seed)
    if mode == "random":
        return rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    out = bytearray()
    step = 1 << 27  # generate in 256 MiB pieces (float32 temporaries)
    while len(out) < nbytes:
        n = min(step, (nbytes - len(out)) // 2)
        w = rng.standard_normal(n).astype(np.float32) * 0.02
        out += (w.view(np.uint32) >> 16).astype(np.uint16).tobytes()
        if n == 0:
            out += b"\0" * (nbytes - len(out))
    return bytes(out)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=4096)
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--mode", default="bf16", choices=["bf16", "random"])
    ap.add_argument("--seeders", type=int, default=1)
    ap.add_argument("--verify-bytes", action="store_true", help="also compare every snapshot byte for byte")
    ap.add_argument("--gpu-env", default="", help="extra env for the GPU CLI runs, e.g. ZEST_GPU_STAGING_MB=256")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    shard = a.mb * 1_000_000 // a.shards
    files = {f"model-{i:05d}-of-{a.shards:05d}.safetensors": weights(a.mode, shard, i) for i in range(1, a.shards + 1)}
    files["config.json"] = b'{"model_type": "llama"}'
    total = sum(len(v) for v in files.values())
    hub = FakeHub(policy="bg4" if a.mode == "bf16" else "none", max_xorb_bytes=64 << 20)
    hub.start()
    work = Path(tempfile.mkdtemp(prefix="zest-clipeer-"))
    nodes = []
    res = {"bytes": total, "mode": a.mode, "shards": a.shards, "seeders": a.seeders,
           "source": "warm `zest serve` seeders (xorb cache, page cache) over BEP XET on loopback"}
    try:
        t0 = time.time()
        commit = hub.add_repo("org/clipeer", files, xet_min_size=1000)
        res["publish_s"] = round(time.time() - t0, 2)
        seeders = [Node(hub, work, "s0")]
        nodes += seeders
        seeders[0].run("pull", "org/clipeer", "--no-p2p", "--no-serve", timeout=3600)
        for k in range(1, a.seeders):
            s = Node(hub, work, f"s{k}")
            shutil.copytree(seeders[0].root / "zest" / "xorbs", s.root / "zest" / "xorbs")
            seeders.append(s)
            nodes.append(s)
        for s in seeders:
            s.spawn("serve", "--listen-port", str(s.listen_port), "--http-port", str(s.http_port))
        for s in seeders:
            s.wait_healthy(timeout=30)
        peers = []
        for s in seeders:
            peers += ["--peer", f"127.0.0.1:{s.listen_port}"]
        stored = sum(p.stat().st_size for p in seeders[0].xorb_files())
        res["stored_bytes"] = stored

        gpu_env = dict(kv.split("=", 1) for kv in a.gpu_env.split(",") if kv)
        res["gpu_env"] = gpu_env

        def run(label, extra, env=None):
            t = time.time()
            os.sync()
            synced = time.time() - t
            leech = Node(hub, work, f"leech_{label}")
            nodes.append(leech)
            t1 = time.time()
            r = leech.run("pull", "org/clipeer", "--no-dht", "--no-serve", *peers, *extra, timeout=3600, env=env)
            dt = time.time() - t1
            ratio = p2p_ratio(r.stdout) if "P2P ratio:" in r.stdout else None
            if a.verify_bytes:
                assert_snapshot(leech, "org/clipeer", commit, files)
            res[label] = {"seconds": round(dt, 3), "GBps": round(total / dt / 1e9, 3), "p2p_ratio": ratio,
                          "presync_s": round(synced, 3),
                          "worker": [ln for ln in r.stdout.splitlines() if ln.startswith("[gpu")][-3:]}
            print(f"[{label}] {total / dt / 1e9:.2f} GB/s ({dt:.2f}s), P2P {ratio}", flush=True)
            shutil.rmtree(leech.root, ignore_errors=True)

        run("warmup", [])  # untimed in the result: brings the seeder's cache files into the page cache
        run("host", [])
        run("gpu_cli", ["--gpus", "1"], gpu_env)
        run("host_again", [])
        run("gpu_cli_again", ["--gpus", "1"], gpu_env)
        host = min(res["host"]["seconds"], res["host_again"]["seconds"])
        gpu = min(res["gpu_cli"]["seconds"], res["gpu_cli_again"]["seconds"])
        res["gpu_vs_host"] = round(host / gpu, 3)
        print(json.dumps(res), flush=True)
        if a.out:
            Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
        return 0
    finally:
        for n in nodes:
            n.close()
        hub.stop()
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    raise SystemExit(main())
