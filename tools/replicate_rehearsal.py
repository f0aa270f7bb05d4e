#!/usr/bin/env python3
"""Rehearsal of the single-command replicated pull on a one-GPU box:

    python tools/replicate_rehearsal.py --ranks 2 [--model gpt2]

Publishes a synthetic model on an in-process fake hub (CDN + CAS), then runs
`python -m zest_amd pull <repo> --gpus N --device all --backend gloo --save-snapshot` as ONE child
command (the ranks share the GPU; gloo control plane, peer-mapped exchanges), checks that every
rank reported every tensor and that the snapshot rank 0 wrote matches the published bytes, and
prints one JSON line.  This process never touches the GPU (the hub builds the world on the host).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--mode", default="bf16")
    ap.add_argument("--timeout", type=float, default=240)
    a = ap.parse_args()
    from zest_amd import models
    from zest_amd.synthetic import SyntheticWorld
    from zest_amd.testing import FakeHub

    world = SyntheticWorld(models.get(a.model), seed=5, mode=a.mode)
    hub = FakeHub(policy="auto", max_xorb_bytes=64 << 20)
    hub.start()
    tmp = tempfile.mkdtemp(prefix="zest-replicate-rehearsal-")
    try:
        hub.add_world(world)
        env = dict(os.environ, PYTHONPATH=ROOT)
        env.update(hub.env(tmp))
        cmd = [sys.executable, "-m", "zest_amd", "pull", world.spec.repo_id, "--gpus", str(a.ranks), "--device", "all",
               "--backend", "gloo", "--save-snapshot", "--no-p2p", "--no-dht", "--timeout", str(a.timeout)]
        t0 = time.time()
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=a.timeout + 60)
        wall = time.time() - t0
        sys.stderr.write(r.stdout + r.stderr)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("[rank ")]
        ok = r.returncode == 0 and len(lines) == a.ranks and all("verified" in ln for ln in lines)
        snap_ok = None
        if ok:
            import glob
            snap_ok = True
            for f in world.files:
                hits = glob.glob(os.path.join(tmp, "hf", "**", "snapshots", "*", f.path), recursive=True)
                snap_ok &= bool(hits) and open(hits[0], "rb").read() == world.file_bytes_host(f)
        print(json.dumps({"ranks": a.ranks, "model": world.spec.repo_id, "model_bytes": world.model_bytes, "rc": r.returncode,
                          "status_lines": lines, "snapshot_matches": snap_ok, "wall_s": round(wall, 2)}), flush=True)
        return 0 if ok and snap_ok else 1
    finally:
        hub.stop()


if __name__ == "__main__":
    sys.exit(main())
