#!/usr/bin/env python3
"""Diagnostic: per-step times of the headline pull (bench.py's pipeline) over many steps, to see
whether a long run slows down and where (H2D copies vs kernels).  One GPU.

    python tools/step_times.py --steps 25 [--model llama-3.1-70b]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from zest_amd import models, ops  # noqa: E402
from zest_amd.engine import DevicePuller  # noqa: E402
from zest_amd.parallel import bind_local_numa  # noqa: E402
from zest_amd.synthetic import SyntheticWorld  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--model", default="llama-3.1-70b")
    ap.add_argument("--round-mb", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=0,
                    help="also time runs of this many back-to-back steps (no host sync between steps)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cpus = bind_local_numa(dev)
    world = SyntheticWorld(models.get(a.model), seed=0, mode="random")
    arena = ops.padded_empty(world.arena_bytes, dev)
    world.generate_on_device(arena)
    world.build_on_device(arena)
    puller = DevicePuller(world, arena, 0, 1, round_bytes=a.round_mb << 20)
    puller.build_origin()
    torch.cuda.synchronize()
    H = ops.hip()
    # pure H2D of the same origin spans, for comparison
    stage = ops.padded_empty(max(r.span_len for r in puller.rounds), dev)
    times = []
    step = puller.step
    for k in range(a.steps):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        st = torch.cuda.current_stream().cuda_stream
        for r in puller.rounds:
            H.memcpy_async(stage.data_ptr(), puller.origin.ptr + r.span_off, r.span_len, st)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        times.append({"step": k, "pull_s": round(t1 - t0, 4), "h2d_only_s": round(t2 - t1, 4),
                      "GBps": round(world.model_bytes / (t1 - t0) / 1e9, 2)})
        print(json.dumps(times[-1]), flush=True)
    for nb, ahead in [(a.batch, x) for x in (0, 1)] if a.batch else []:
        puller.steps_ahead = ahead
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(nb):
                puller.step()
            t_issue = time.perf_counter() - t0
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"back_to_back_steps": nb, "steps_ahead": ahead, "rep": rep, "s_per_step": round(dt / nb, 4),
                              "host_issue_s_per_step": round(t_issue / nb, 4),
                              "GBps": round(nb * world.model_bytes / dt / 1e9, 2)}), flush=True)
    puller.check()
    print(json.dumps({"numa_cpus": len(cpus), "origin_bytes": puller.origin.n}), flush=True)


if __name__ == "__main__":
    main()
