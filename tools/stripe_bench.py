"""Host `zest pull` throughput from 1 vs 3 warm loopback seeders (term striping).

Every "machine" is a cache root + port set on 127.0.0.1 (tests/e2e_util.Node).  Seeder 0 pulls the
repo from the fake CDN; seeders 1-2 get a copy of its xorb cache; all three run `zest serve`.  A
fresh leecher then pulls with `--peer` = seeder 0 only, and another with all three.  Reports wall
time, GB/s and each seeder's share of the bytes served (from its /v1/status).

    python tools/stripe_bench.py [--mb 2048] [--out profiles/stripe_bench.json]

Reference target: "Lab with 5 warm peers: 15 sec (parallel LAN), 20x" (DESIGN.md:570); the
reference itself tries peers sequentially, first success wins (swarm.zig:371-394).
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import shutil
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from e2e_util import Node, p2p_ratio  # noqa: E402
from zest_amd.testing import FakeHub  # noqa: E402


def _proc_cpu(pid: int) -> float:
    """CPU seconds (user + system) of a live process."""
    try:
        with open(f"/proc/{pid}/stat") as fh:
            f = fh.read().rsplit(")", 1)[1].split()
        return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, IndexError):
        return 0.0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=2048, help="repo size (MB of random weights, 4 shards)")
    ap.add_argument("--shards", type=int, default=4, help="number of weight files the repo is split into")
    ap.add_argument("--out", default=None)
    ap.add_argument("--trace", default=None, help="directory: each leecher writes a ZEST_TRACE Chrome trace there")
    ap.add_argument("--rate-mbps", type=float, default=0.0,
                    help="cap each seeder's uplink (zest serve --fault rate:<MB/s>, shared by its connections): "
                         "1250 ~ a 10 Gbps LAN peer")
    ap.add_argument("--jobs", type=int, default=0, help="leecher --concurrency (default: the CLI's 16)")
    a = ap.parse_args()
    if a.trace:
        Path(a.trace).mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(1)
    shard = a.mb * 1_000_000 // a.shards
    files = {f"model-{i:05d}-of-{a.shards:05d}.safetensors": rng.integers(0, 256, shard, dtype=np.uint8).tobytes()
             for i in range(1, a.shards + 1)}
    files["config.json"] = b'{"model_type": "llama"}'
    total = sum(len(v) for v in files.values())
    hub = FakeHub(policy="none")
    hub.start()
    work = Path(tempfile.mkdtemp(prefix="zest-stripe-"))
    nodes = []
    res = {"bytes": total, "repo": "org/stripe", "data": f"random bytes, {a.shards} Xet shards, raw chunks",
           "seeder_rate_mbps": a.rate_mbps or None, "leech_jobs": a.jobs or 16}
    try:
        hub.add_repo("org/stripe", files, xet_min_size=1000)
        seeders = [Node(hub, work, "s0")]
        nodes += seeders
        seeders[0].run("pull", "org/stripe", "--no-p2p", "--no-serve", timeout=1800)
        for k in (1, 2):
            s = Node(hub, work, f"s{k}")
            shutil.copytree(seeders[0].root / "zest" / "xorbs", s.root / "zest" / "xorbs")
            seeders.append(s)
            nodes.append(s)
        for s in seeders:
            extra = ["--fault", f"rate:{a.rate_mbps}"] if a.rate_mbps > 0 else []
            s.spawn("serve", "--listen-port", str(s.listen_port), "--http-port", str(s.http_port), *extra)
        for s in seeders:
            s.wait_healthy(timeout=30)
        for label, use in (("1_seeder", seeders[:1]), ("3_seeders", seeders)):
            st0 = [json.loads(s.api("/v1/status")[1]) for s in seeders]
            before = [x["bytes_served"] for x in st0]
            leech = Node(hub, work, f"leech_{label}")
            nodes.append(leech)
            args = ["pull", "org/stripe", "--no-dht", "--no-serve"] + (["-j", str(a.jobs)] if a.jobs else [])
            for s in use:
                args += ["--peer", f"127.0.0.1:{s.listen_port}"]
            scpu0 = [_proc_cpu(s.procs[-1].pid) for s in seeders]
            lcpu0 = resource.getrusage(resource.RUSAGE_CHILDREN)
            t0 = time.time()
            env = {"ZEST_TRACE": str(Path(a.trace).resolve() / f"leech_{label}.json")} if a.trace else None
            r = leech.run(*args, timeout=1800, env=env)
            dt = time.time() - t0
            lcpu1 = resource.getrusage(resource.RUSAGE_CHILDREN)
            # CPU seconds of the leecher (a finished child) and of each seeder process during the pull
            cpu = {"leecher": round(lcpu1.ru_utime + lcpu1.ru_stime - lcpu0.ru_utime - lcpu0.ru_stime, 3),
                   "seeders": [round(_proc_cpu(s.procs[-1].pid) - c, 3) for s, c in zip(seeders, scpu0)]}
            st1 = [json.loads(s.api("/v1/status")[1]) for s in seeders]
            after = [x["bytes_served"] for x in st1]
            # each seeder's connection-thread seconds in run lookups and socket writes during this pull
            split = {k: [round(b.get(k, 0) - a_.get(k, 0), 3) for a_, b in zip(st0, st1)]
                     for k in ("serve_lookup_s", "serve_wait_s", "serve_send_s")}
            served = [b - a_ for a_, b in zip(before, after)]
            res[label] = {"seconds": round(dt, 3), "GBps": round(total / dt / 1e9, 3), "p2p_ratio": p2p_ratio(r.stdout),
                          "served_share": [round(x / max(1, sum(served)), 3) for x in served], "seeders": split,
                          "cpu_s": cpu, "cpus_busy": round((cpu["leecher"] + sum(cpu["seeders"])) / dt, 2)}
            if a.trace:  # the peer-transfer phase alone (first request start .. last response end)
                ev = json.load(open(Path(a.trace) / f"leech_{label}.json"))
                ev = ev["traceEvents"] if isinstance(ev, dict) else ev
                req = [e for e in ev if e.get("ph") == "X" and e.get("cat") == "peer" and e.get("name") == "request"]
                tot: dict = {}
                for e in ev:  # where the leecher's threads spent their time (summed over threads)
                    if e.get("ph") == "X":
                        k = f"{e.get('cat')}/{e.get('name')}"
                        tot[k] = tot.get(k, 0.0) + e.get("dur", 0) / 1e3
                res[label]["span_ms"] = {k: round(v, 1) for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]}
                if req:
                    span = (max(e["ts"] + e["dur"] for e in req) - min(e["ts"] for e in req)) / 1e6
                    res[label]["transfer_s"] = round(span, 3)
                    res[label]["transfer_GBps"] = round(total / span / 1e9, 3)
            print(f"[{label}] {total / dt / 1e9:.2f} GB/s ({dt:.1f}s), P2P {p2p_ratio(r.stdout):.0f}%, "
                  f"seeder shares {res[label]['served_share']}", flush=True)
        res["speedup_3_vs_1"] = round(res["1_seeder"]["seconds"] / res["3_seeders"]["seconds"], 3)
        if "transfer_s" in res["3_seeders"]:
            res["transfer_speedup_3_vs_1"] = round(res["1_seeder"]["transfer_s"] / res["3_seeders"]["transfer_s"], 3)
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
