"""BASELINE config 4: `zest pull Qwen/Qwen2-7B --revision v1.0` with peer discovery via DHT and the
BT tracker (the BEP XET path, no --peer).

Scenario (all on loopback, offline fake Hub + tracker, synthetic random-byte weights with the real
Qwen2-7B tensor shapes):
  1. a DHT bootstrap node starts;
  2. the seeder pulls the repo CDN-only, then runs `zest seed --tracker ... --dht-bootstrap ...`,
     announcing every cached xorb's info_hash to both;
  3. the leecher runs `zest pull <repo> --revision v1.0 --tracker ... --dht-bootstrap ...` and must
     find the seeder itself.
Prints one JSON line: bytes, seconds, GB/s and P2P ratio for the CDN pull and for the discovered
P2P pull, and the number of announces the tracker and the DHT saw.

    python tools/discovery_bench.py [--model qwen2-7b] [--out profiles/discovery_qwen2_7b.json]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from e2e_util import ZEST, free_port  # noqa: E402
from zest_amd import _core, models  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402
from zest_amd.testing import FakeHub  # noqa: E402


def node_env(hub: FakeHub, root: Path) -> dict:
    env = dict(os.environ, **hub.env(str(root)))
    env["ZEST_LISTEN_PORT"] = str(free_port())
    env["ZEST_HTTP_PORT"] = str(free_port())
    return env


def timed(cmd, env, timeout=3600):
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    dt = time.time() - t0
    if r.returncode != 0:
        raise SystemExit(f"{' '.join(cmd)} failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
    return r.stdout, dt


def ratio(out: str) -> float:
    m = re.findall(r"P2P ratio:\s*([0-9.]+)", out)
    return float(m[-1]) if m else 0.0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2-7b")
    ap.add_argument("--revision", default="v1.0")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    spec = models.get(a.model)
    t0 = time.time()
    world = SyntheticWorld(spec, seed=3, max_xorb_bytes=64 << 20)
    hub = FakeHub(policy="none", max_xorb_bytes=64 << 20)
    commit = hub.add_world(world, revision=a.revision, exact=True)
    url = hub.start()
    total = sum(f.size for f in world.files)
    print(f"[setup] {spec.repo_id}@{a.revision}: {total / 1e9:.2f} GB, {len(hub.xorbs)} xorbs "
          f"({time.time() - t0:.1f}s)", flush=True)
    tracker = url + "/announce"
    boot = _core.dht.Node(0)
    bs = f"127.0.0.1:{boot.port}"
    work = Path(tempfile.mkdtemp(prefix="zest-disc-"))
    seed_proc = None
    try:
        # 1. seeder: CDN pull, then seed (announce to tracker + DHT)
        senv = node_env(hub, work / "seeder")
        out, cdn_s = timed([str(ZEST), "pull", spec.repo_id, "--revision", a.revision, "--no-p2p"], senv)
        print(f"[seeder] CDN pull {total / cdn_s / 1e9:.2f} GB/s ({cdn_s:.1f}s)", flush=True)
        s_listen, s_dht = free_port(), free_port(2)
        seed_proc = subprocess.Popen([str(ZEST), "seed", "--tracker", tracker, "--dht-bootstrap", bs, "--dht-port",
                                      str(s_dht), "--listen", str(s_listen)], env=senv, stdout=subprocess.PIPE,
                                     stderr=subprocess.STDOUT, text=True)
        ihs = [_core.info_hash(_core.from_xet_hex(x.hash_hex)) for x in hub.xorbs]
        t_ann = time.time()
        while time.time() - t_ann < 120:
            if hub.counters.get("announce", 0) >= len(ihs) and all(boot.stored_peers(ih) for ih in ihs):
                break
            time.sleep(0.2)
        ann_s = time.time() - t_ann
        n_dht = sum(1 for ih in ihs if boot.stored_peers(ih))
        print(f"[seeder] announced {hub.counters.get('announce', 0)} to tracker, {n_dht}/{len(ihs)} in DHT "
              f"({ann_s:.1f}s)", flush=True)
        # 2. leecher: discovery only (no --peer)
        lenv = node_env(hub, work / "leecher")
        xorb_gets = hub.counters.get("xorb_get", 0)
        out, p2p_s = timed([str(ZEST), "pull", spec.repo_id, "--revision", a.revision, "--tracker", tracker,
                            "--dht-bootstrap", bs, "--dht-port", str(free_port(2))], lenv)
        r = ratio(out)
        cdn_after = hub.counters.get("xorb_get", 0) - xorb_gets
        print(f"[leecher] discovered P2P pull {total / p2p_s / 1e9:.2f} GB/s ({p2p_s:.1f}s), P2P ratio {r}%, "
              f"{cdn_after} CDN xorb GETs", flush=True)
        snap = work / "leecher" / "hf" / "hub" / ("models--" + spec.repo_id.replace("/", "--")) / "snapshots" / commit
        ok = all((snap / f.path).stat().st_size == f.size for f in world.files)
        res = {"scenario": f"{spec.repo_id} --revision {a.revision} via DHT + tracker (bep_xet)", "model": a.model,
               "bytes": total, "xorbs": len(hub.xorbs), "cdn_pull_s": round(cdn_s, 3),
               "cdn_pull_gbps": round(total / cdn_s / 1e9, 3), "p2p_pull_s": round(p2p_s, 3),
               "p2p_pull_gbps": round(total / p2p_s / 1e9, 3), "p2p_ratio": r, "cdn_xorb_gets_during_p2p": cdn_after,
               "tracker_announces": hub.counters.get("announce", 0), "dht_swarms": n_dht, "snapshot_ok": ok,
               "data": "synthetic random-byte weights, real tensor shapes; loopback, offline fake Hub"}
        print(json.dumps(res), flush=True)
        if a.out:
            Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
        return 0 if ok and r > 0 else 1
    finally:
        if seed_proc is not None:
            seed_proc.terminate()
            seed_proc.wait(timeout=30)
        boot.stop()
        hub.stop()
        subprocess.run(["rm", "-rf", str(work)])


if __name__ == "__main__":
    raise SystemExit(main())
