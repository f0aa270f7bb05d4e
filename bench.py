#!/usr/bin/env python3
"""Headline benchmark: aggregate pull GB/s + P2P ratio, Llama-3.1-70B, N MI355X peers (BASELINE.json).

One process per GPU (torchrun for N > 1; RCCL = torch.distributed "nccl").  Every rank ends each
step holding the complete, Merkle-verified model (141 GB of bf16 weights in 30 safetensors shards)
in its HBM arena:

  origin (pinned host, = the CDN bytes of this rank's 1/N of the reconstruction terms)
    --hipMemcpyAsync--> HBM staging ring --HIP index/place/BLAKE3--> arena
    --RCCL / IPC over xGMI--> every other GPU, which BLAKE3-hashes what it received as each round
    lands; GPU Merkle file hashes on every rank against the published ones.

The replication strategy (batched RCCL p2p sends, coalesced broadcasts, equal-slab all-gather, DMA
copies from the peers' IPC-mapped arenas, or the K8 gather kernel reading every peer at once over
xGMI) is picked during setup by timing each one on the machine (--exchange auto,
DevicePuller.autotune_exchange).

value      = N * model_bytes / step_time   (bytes made resident + verified across all GPUs, GB/s)
p2p_ratio  = fraction of each GPU's model bytes that arrived from peers rather than the origin
Data: synthetic (random-byte weights of the real Llama-3.1-70B tensor shapes; CDC/xorbs/hashes
built with the real Xet algorithms); no network exists, so the origin is pinned host memory.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--model llama-3.1-70b] ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

BASELINE_METRIC = "aggregate pull GB/s + P2P ratio, Llama-3.1-70B at 1/2/4/8 MI355X peers"


def log(rank, *a):
    if rank == 0 or os.environ.get("ZEST_BENCH_LOG_ALL") == "1":
        print(f"[bench{'' if rank == 0 else f' r{rank}'}]", *a, file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3.1-70b")
    ap.add_argument("--mode", default="random", choices=["random", "bf16"])
    ap.add_argument("--round-mb", type=int, default=1024, help="per-rank bytes per pipeline round")
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--seeders", type=int, default=0,
                    help="ranks that pull from the origin (default all); the rest leech everything from "
                         "them over xGMI (BASELINE config 2: --gpus 2 --seeders 1)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "p2p", "bcast", "allgather", "ipc", "xgmi"],
                    help="intra-node replication strategy; auto = time each on this machine during setup")
    a = ap.parse_args()

    from zest_amd import models, ops
    from zest_amd.engine import DevicePuller
    from zest_amd.synthetic import SyntheticWorld

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != a.gpus:
        if world_size == 1 and a.gpus > 1:
            raise SystemExit("for --gpus > 1 launch with torchrun --nproc-per-node N (one rank per GPU)")
    # ZEST_BENCH_BACKEND=gloo is a rehearsal mode for one-GPU boxes: several ranks share the device,
    # control traffic goes over gloo, and only the peer-mapped exchanges (ipc / xgmi) can move the
    # data.  Its numbers are not xGMI measurements; the JSON line says so in config.backend.
    backend = os.environ.get("ZEST_BENCH_BACKEND", "nccl")
    if os.environ.get("ZEST_BENCH_WATCHDOG"):  # diagnostics: dump every thread's stack and exit
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["ZEST_BENCH_WATCHDOG"]), exit=True)
    device = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank)
    torch.cuda.set_device(device)
    from zest_amd.parallel import bind_local_numa
    numa_cpus = bind_local_numa(device)
    dist = None
    if world_size > 1:
        import torch.distributed as dist
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            from zest_amd.parallel import nccl_options
            dist.init_process_group("nccl", device_id=device, pg_options=nccl_options())
    t_setup = time.time()
    ops.hip()
    spec = models.get(a.model)
    # bf16 mode stores chunks the way Xet stores real checkpoints: BG4-LZ4 frames (compressed on the
    # GPU) when smaller than the chunk, so the pull decodes them on the GPU.
    world = SyntheticWorld(spec, seed=a.seed, mode=a.mode, compression="bg4" if a.mode == "bf16" else "none")
    if numa_cpus:
        log(rank, f"bound to {len(numa_cpus)} CPUs on the GPU's NUMA node")
    log(rank, f"model {spec.repo_id}: {world.model_bytes / 1e9:.2f} GB in {len(world.xet_files)} files; "
              f"arena {world.arena_bytes / 1e9:.2f} GB; ranks {world_size}")
    arena = ops.padded_empty(world.arena_bytes, device)
    world.generate_on_device(arena)
    world.build_on_device(arena)
    torch.cuda.synchronize()
    log(rank, f"xet plan: {world.n_chunks} chunks, {world.n_xorbs} xorbs, {len(world.terms)} terms "
              f"({time.time() - t_setup:.1f}s)")
    # Host oracle spot check of the GPU chunk hashes (8 chunks spread over the model).
    from zest_amd import _core
    for j in np.linspace(0, world.n_chunks - 1, 8).astype(int):
        o, n = int(world.chunk_off[j]), int(world.chunk_len[j])
        assert world.chunk_hashes[j].tobytes() == _core.chunk_hash(arena[o:o + n].cpu().numpy().tobytes()), j
    if dist is not None:
        fp = torch.tensor([int.from_bytes(world.file_hashes[:, :8].tobytes()[:8], "little") & 0x7FFFFFFFFFFFFFFF],
                          dtype=torch.int64, device=device)
        lo, hi = fp.clone(), fp.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        assert int(lo.item()) == int(hi.item()), "ranks disagree on the synthetic repository"
    seeders = a.seeders if a.seeders > 0 else world_size
    puller = DevicePuller(world, arena, rank, world_size, round_bytes=a.round_mb << 20, slots=a.slots,
                          seeders=seeders)
    if world_size > 1:
        # The peer-mapped exchanges are opt-in under auto (ZEST_EXCHANGE_IPC=1): in a 2-rank bench
        # rehearsal on one GPU (tools/gpu_bench_rehearsal.sh) importing a peer's 16 GB arena handle
        # hung inside hipIpcOpenMemHandle, before or after the origin build, while a standalone
        # probe with the same sizes, pinned memory and NUMA binding imports in 1 ms
        # (tools/gpu_ipc_probe2.sh); cause not found yet, and a hang would cost the scaling run.
        want_ipc = a.exchange in ("ipc", "xgmi") or (a.exchange == "auto" and os.environ.get("ZEST_EXCHANGE_IPC") == "1")
        ipc = want_ipc and puller.enable_ipc()
        log(rank, f"peer arenas mapped over HIP IPC: {ipc}")
        if a.exchange in ("ipc", "xgmi") and not ipc:
            raise SystemExit(f"--exchange {a.exchange}: mapping the peers' arenas failed")
    puller.build_origin()
    torch.cuda.synchronize()
    # ZEST_GRAPH=1 (one GPU): a step is one HIP graph launch.  Opt-in: the graph's H2D copies ran at
    # 51.2 GB/s against 56.2 for the eager copy-stream pipeline (profiles/hip_graph_r2.md).
    graph = puller.capture_graph() if world_size == 1 and os.environ.get("ZEST_GRAPH") == "1" else False
    if graph:
        log(rank, "step captured in a HIP graph")
    log(rank, f"origin {puller.origin.n / 1e9:.2f} GB pinned on rank {rank}; rounds {puller.n_rounds}; "
              f"setup {time.time() - t_setup:.1f}s")
    if world_size > 1:
        if a.exchange == "auto":
            t_x = puller.autotune_exchange()
            log(rank, "exchange autotune (s over the first rounds): "
                + ", ".join(f"{m}={v:.3f}" for m, v in t_x.items()) + f" -> {puller.exchange}")
        else:
            puller.exchange = a.exchange

    def barrier():
        if dist is not None:
            dist.barrier()

    # Warm-up steps on a poisoned arena: prove every byte is really placed (every step re-hashes every
    # chunk of every replica, so a faulty exchange strategy shows up here as a hash mismatch).
    def warmup():
        for _ in range(a.warmup):
            arena.fill_(0xA5)
            puller.err.zero_()
            puller.step()
            torch.cuda.synchronize()
            puller.check()

    try:
        warmup()
    except ops.IngestError as e:  # the error word is all-reduced: every rank takes this branch
        if world_size == 1 or puller.exchange == "p2p":
            raise
        log(rank, f"exchange {puller.exchange} failed verification ({e}); falling back to p2p")
        puller.exchange = "p2p"
        warmup()
    puller.err.zero_()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        puller.step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    puller.check()  # all timed steps verified (first error persists)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    step_s = float(elapsed.item()) / max(1, a.steps)
    model_b = world.model_bytes
    value = world_size * model_b / step_s / 1e9
    recv = torch.tensor([float(puller.bytes_received)], dtype=torch.float64, device=device)
    ing = torch.tensor([float(puller.bytes_ingested)], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(recv)
        dist.all_reduce(ing)
    p2p_ratio = float(recv.item()) / (world_size * model_b)
    out = {
        "metric": BASELINE_METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(step_s * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": f"synthetic ({a.mode}-byte weights of the real tensor shapes; real Xet CDC/xorbs/hashes"
                + ("; BG4-LZ4 compressed chunks, stored/raw ratio "
                   f"{float(world.chunk_clen.sum()) / float(world.chunk_len.sum()):.3f}" if a.mode == "bf16" else "")
                + "; origin = pinned host memory standing in for the CDN)",
        "p2p_ratio": round(p2p_ratio, 4),
        "ingest_GBps": round(float(ing.item()) / step_s / 1e9, 3),
        "config": {"model": spec.repo_id, "global_batch": world_size, "seq_len": None,
                   "parallelism": (f"swarm{world_size}" if seeders == world_size
                                   else f"seed{seeders}-leech{world_size - seeders}"), "model_bytes": model_b, "files": len(world.xet_files),
                   "chunks": world.n_chunks, "xorbs": world.n_xorbs, "terms": int(len(world.terms)),
                   "rounds": puller.n_rounds, "round_mb": a.round_mb, "exchange": puller.exchange if world_size > 1 else "none",
                   "exchange_autotune_s": {m: round(v, 4) for m, v in puller.exchange_times.items()},
                   "verify": "blake3 of every chunk on every rank + merkle file hashes",
                   "numa_bound_cpus": len(numa_cpus), "hip_graph": bool(graph),
                   "pipeline": getattr(puller, "pipeline", "cpu"),
                   "backend": backend if world_size > 1 else "none"},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    puller.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
