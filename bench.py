#!/usr/bin/env python3
"""Headline benchmark: aggregate pull GB/s + P2P ratio, Llama-3.1-70B, N MI355X peers (BASELINE.json).

One process per GPU (RCCL = torch.distributed "nccl").  Every rank ends each step holding the
complete, Merkle-verified model (141 GB of bf16 weights in 30 safetensors shards) in its HBM arena:

  origin (pinned host, = the CDN bytes of this rank's 1/N of the reconstruction terms)
    --hipMemcpyAsync--> HBM staging ring --HIP index/place|LZ4-BG4 decode/BLAKE3--> arena
    --RCCL / IPC over xGMI--> every other GPU, which BLAKE3-hashes what it received as each round
    lands; GPU Merkle file hashes on every rank against the published ones.

Data modes (--modes, first = the headline `value`, the others are reported under `extra`):
  bf16    N(0, 0.02) bf16 weights stored the way Xet stores real checkpoints: BG4-LZ4 chunk frames
          when smaller than the chunk (stored/raw ~0.88), so every step decodes them on the GPU.
  random  uniformly random bytes (incompressible; stored raw, as Xet does).

value      = N * model_bytes / step_time   (bytes made resident + verified across all GPUs, GB/s)
p2p_ratio  = fraction of each GPU's model bytes that arrived from peers rather than the origin
No network exists, so the origin is pinned host memory standing in for the CDN.

Launch: `python bench.py --gpus N` starts torchrun itself for N > 1 (a child process; rank 0's JSON
line is forwarded and the child's exit status returned); under torchrun (WORLD_SIZE set) it runs
as one rank.  At N > 1 a watchdog bounds every phase (faulthandler stack dump, then exit 1), and the
process group has an explicit timeout, so a stuck collective ends the run with a stack instead of
an empty record.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--model llama-3.1-70b] [--modes bf16,random]
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

BASELINE_METRIC = "aggregate pull GB/s + P2P ratio, Llama-3.1-70B at 1/2/4/8 MI355X peers"
HEADLINE_REPO = "meta-llama/Llama-3.1-70B"


def metric_name(spec) -> str:
    """BASELINE.json's metric for the headline model; any other model is named as what it is."""
    if spec.repo_id == HEADLINE_REPO:
        return BASELINE_METRIC
    return (f"aggregate pull GB/s + P2P ratio, {spec.repo_id.split('/')[-1]} at 1/2/4/8 MI355X peers "
            f"(not the headline config: {HEADLINE_REPO.split('/')[-1]})")
MODES = ("bf16", "random")

# Per-phase watchdog limits (seconds) for N > 1; ZEST_BENCH_WATCHDOG=<s> overrides all, =0 disables.
# "1": --exchange auto also maps the peers' arenas (HIP VMM, dmabuf fds) and times the ipc / xgmi
# exchanges next to the RCCL ones; a mapping that fails, times out or does not read back falls back
# to RCCL.  ZEST_EXCHANGE_IPC=0 turns it off.
IPC_AUTO = "1"
PHASE_LIMITS = {"init": 180, "setup": 420, "ipc": 90, "autotune": 180, "warmup": 240, "timed": 420,
                "report": 120, "swarm_setup": 180, "swarm_warmup": 300, "swarm_timed": 300, "swarm_report": 120}


def log(rank, *a):
    if rank == 0 or os.environ.get("ZEST_BENCH_LOG_ALL") == "1":
        print(f"[bench{'' if rank == 0 else f' r{rank}'}]", *a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3.1-70b")
    ap.add_argument("--modes", default=",".join(MODES),
                    help="comma list of data modes; the first is the headline value, the rest go in extra")
    ap.add_argument("--mode", default=None, choices=list(MODES), help="single data mode (= --modes MODE)")
    ap.add_argument("--round-mb", type=int, default=1024, help="per-rank bytes per pipeline round")
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--seeders", type=int, default=0,
                    help="ranks that pull from the origin (default all); the rest leech everything from "
                         "them over xGMI (BASELINE config 2: --gpus 2 --seeders 1)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "p2p", "bcast", "allgather", "ipc", "xgmi"],
                    help="intra-node replication strategy; auto = time each on this machine during setup")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo rehearsal of the whole bench on host memory (tests; not a GPU number)")
    ap.add_argument("--swarm-row", default="auto", choices=["auto", "on", "off"],
                    help="also time the PUBLIC path, zest_amd.parallel.swarm_pull (= pull(device='all')), on the "
                         "last data mode's world, its CDN served from the same pinned origin through an "
                         "in-process memory CAS (mem:// fetch_info URLs, no sockets); reported under "
                         "extra.swarm_pull_*.  auto: on for GPU runs (at N > 1 a failure or overrun of the row is "
                         "recorded in extra.swarm_pull_error and never costs the headline line)")
    ap.add_argument("--swarm-steps", type=int, default=2)
    ap.add_argument("--swarm-warmup", type=int, default=1)
    a = ap.parse_args(argv)
    a.modes = [a.mode] if a.mode else [m for m in a.modes.split(",") if m]
    bad = [m for m in a.modes if m not in MODES]
    if bad or not a.modes:
        ap.error(f"--modes: unknown {bad}; choose from {list(MODES)}")
    return a


# ------------------------------------------------------------------------------------------------
# N > 1 without torchrun: this process becomes a launcher (before anything touches the GPU)
# ------------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str], timeout_s: float | None = None) -> int:
    """Run this script under torchrun with n ranks as a child process group; returns its exit code
    (124 when it exceeded `timeout_s`, after the whole group was killed)."""
    port = os.environ.get("ZEST_BENCH_PORT") or str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return proc.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        print(f"[bench] ranks exceeded {timeout_s:.0f}s; killing the process group", file=sys.stderr, flush=True)
        for sig, grace in ((signal.SIGTERM, 10), (signal.SIGKILL, 10)):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                break
            try:
                proc.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        return 124
    except KeyboardInterrupt:
        os.killpg(proc.pid, signal.SIGTERM)
        proc.wait()
        return 130


class Watchdog:
    """Per-phase deadline: faulthandler dumps every thread's stack and exits the rank (torchrun then
    tears the other ranks down).  Off at N = 1 unless ZEST_BENCH_WATCHDOG is set."""

    def __init__(self, rank: int, enabled: bool):
        v = os.environ.get("ZEST_BENCH_WATCHDOG", "")
        self.override = float(v) if v not in ("", "0") else None
        self.enabled = (enabled and v != "0") or self.override is not None
        self.rank = rank
        # Set while an optional row runs after the headline is measured (the N > 1 swarm row): a
        # phase that overruns then calls fallback(reason) -- rank 0 prints the headline line with the
        # row marked failed -- and the rank exits 0, instead of losing the headline with the row.
        self.fallback = None
        self._timer = None

    def _cancel(self) -> None:
        import faulthandler
        faulthandler.cancel_dump_traceback_later()
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None

    def _expire(self, phase: str, limit: float) -> None:
        import faulthandler
        print(f"[bench] watchdog: phase {phase} exceeded {limit:.0f}s; stacks follow", file=sys.stderr, flush=True)
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        try:
            self.fallback(f"phase {phase} exceeded {limit:.0f}s")
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)

    def arm(self, phase: str) -> None:
        if self.enabled:
            import faulthandler
            limit = self.override or PHASE_LIMITS[phase]
            self._cancel()
            log(self.rank, f"watchdog: phase {phase}, {limit:.0f}s")
            if self.fallback is None:
                faulthandler.dump_traceback_later(limit, exit=True)
            else:
                self._timer = threading.Timer(limit, self._expire, args=(phase, limit))
                self._timer.daemon = True
                self._timer.start()
        if os.environ.get("ZEST_BENCH_FAULT") == f"hang:{self.rank}:{phase}":  # fault injection (tests)
            time.sleep(1e9)

    def disarm(self) -> None:
        if self.enabled:
            self._cancel()


# ------------------------------------------------------------------------------------------------
# One rank
# ------------------------------------------------------------------------------------------------
def run_mode(a, mode, spec, device, rank, world_size, dist, wd, exchange_pick=None, arenas=None, keep=None) -> dict:
    """Build the synthetic world of one data mode, pull it a.warmup + a.steps times; returns the
    measured numbers (every rank) plus the puller's exchange choice."""
    import numpy as np
    import torch

    from zest_amd import ops
    from zest_amd.engine import DevicePuller
    from zest_amd.synthetic import SyntheticWorld

    cuda = device.type == "cuda"
    # The peer-mapped exchanges (ipc DMA copies / xgmi K8 kernel) are tried under auto too; a failed
    # or timed-out mapping falls back to the RCCL exchanges.  ZEST_EXCHANGE_IPC=0 turns them off.
    want_ipc = world_size > 1 and cuda and (
        a.exchange in ("ipc", "xgmi") or (a.exchange == "auto" and os.environ.get("ZEST_EXCHANGE_IPC", IPC_AUTO) != "0"))
    mapped = arenas.get("peers") if arenas is not None else None
    wd.arm("setup")
    t_setup = time.time()
    phase: dict = {}
    # bf16 mode stores chunks the way Xet stores real checkpoints: BG4-LZ4 frames (compressed on the
    # GPU) when smaller than the chunk, so the pull decodes them on the GPU.
    comp = "bg4" if (mode == "bf16" and cuda) else "none"
    world = SyntheticWorld(spec, seed=a.seed, mode=mode, compression=comp)
    log(rank, f"[{mode}] model {spec.repo_id}: {world.model_bytes / 1e9:.2f} GB in {len(world.xet_files)} files; "
              f"arena {world.arena_bytes / 1e9:.2f} GB; ranks {world_size}")
    contents = None
    if cuda:
        # One arena for every data mode (the layout depends only on the model's files): freeing and
        # re-allocating 141 GB between modes is avoidable churn in the HBM allocator.
        if arenas is not None and arenas.get("arena") is not None and arenas["arena"].numel() == world.arena_bytes:
            arena = arenas["arena"]
        else:
            arena = None
            if want_ipc:  # a HIP VMM arena: the peers map it through dmabuf fds (csrc/bind/hip_vmm.cpp)
                try:
                    arena = ops.vmm_empty(world.arena_bytes, device)
                except Exception as e:  # noqa: BLE001
                    log(rank, f"VMM arena unavailable ({e}); torch allocation")
            if arena is None:
                arena = ops.padded_empty(world.arena_bytes, device)
            if arenas is not None:
                arenas["arena"] = arena
            if want_ipc:
                # map the peers' arenas while they are fresh allocations, before any kernel wrote
                # them (imports of a built arena were seen to hang, docs/PARITY.md)
                from zest_amd.engine import map_peer_arenas
                wd.arm("ipc")
                t_map = time.time()
                mapped = map_peer_arenas(arena, rank, world_size)
                phase["map_s"] = round(time.time() - t_map, 3)
                wd.arm("setup")
                if arenas is not None:
                    arenas["peers"] = mapped
                log(rank, f"peer arenas mapped over HIP IPC before the build: {mapped is not None}")
        world.generate_on_device(arena)
        # One rank, compressed world: the build's compression writes the serialized chunks straight
        # into pinned memory that becomes the origin (no second compression pass in build_origin).
        ser_store = None
        if comp == "bg4" and world_size == 1:
            from zest_amd.engine import pinned_take
            cap, ptr = pinned_take(int(world.model_bytes * 1.002) + (256 << 20))
            ser_store = (ptr, cap)
        # N > 1: each rank chunks / hashes / compresses only its files, then the plan is all-gathered
        world.build_on_device(arena, shard=(rank, world_size, None) if dist is not None else None,
                              ser_store=ser_store)
        torch.cuda.synchronize()
        if ser_store is not None and world.serialized is None:
            from zest_amd.engine import pinned_give
            pinned_give(ser_store[1], ser_store[0])
    else:
        contents = world.build_on_host()
        arena = torch.zeros(world.arena_bytes + 4096, dtype=torch.uint8)[: world.arena_bytes]
    phase["world_s"] = round(time.time() - t_setup - phase.get("map_s", 0.0), 3)
    log(rank, f"[{mode}] xet plan: {world.n_chunks} chunks, {world.n_xorbs} xorbs, {len(world.terms)} terms "
              f"({time.time() - t_setup:.1f}s)")
    if cuda:  # host oracle spot check of the GPU chunk hashes (8 chunks spread over the model)
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
    # Pin once for every data mode: the origin of a raw world is the largest (+8 B per chunk header),
    # and a share is within one 64 MiB xorb term of 1/seeders of it.
    reserve = (int(world.model_bytes * 1.002) // seeders + (256 << 20)) if rank < seeders else 0
    puller = DevicePuller(world, arena, rank, world_size, round_bytes=a.round_mb << 20, slots=a.slots,
                          seeders=seeders, origin_reserve=reserve)
    if getattr(world, "serialized", None) is not None:  # not adopted: back to the pool
        from zest_amd.engine import pinned_give
        pinned_give(world.serialized[1], world.serialized[0])
        world.serialized = None
    phase["origin_adopted"] = bool(getattr(puller, "origin_prebuilt", False))
    ipc = False
    if want_ipc:
        ipc = mapped is not None and puller.enable_ipc(mapped)
        if a.exchange in ("ipc", "xgmi") and not ipc:
            raise SystemExit(f"--exchange {a.exchange}: mapping the peers' arenas failed")
    t_origin = time.time()
    if cuda:
        puller.build_origin()
        torch.cuda.synchronize()
    else:
        puller.build_origin_host(contents)
    phase["origin_s"] = round(time.time() - t_origin, 3)
    # ZEST_GRAPH=1 (one GPU): a step is one HIP graph launch.  Opt-in: the graph's H2D copies ran at
    # 51.2 GB/s against 56.2 for the eager copy-stream pipeline (profiles/hip_graph_r2.md).
    graph = puller.capture_graph() if world_size == 1 and os.environ.get("ZEST_GRAPH") == "1" else False
    if graph:
        log(rank, "step captured in a HIP graph")
    log(rank, f"[{mode}] origin {puller.origin.n / 1e9:.2f} GB pinned on rank {rank}; rounds {puller.n_rounds}; "
              f"setup {time.time() - t_setup:.1f}s")
    phase["setup_s"] = round(time.time() - t_setup, 3)
    t_tune = time.time()
    if world_size > 1:
        wd.arm("autotune")
        if exchange_pick is not None and (exchange_pick not in ("ipc", "xgmi") or ipc):
            puller.exchange = exchange_pick  # chosen on the first mode's world (same plan shape)
        elif a.exchange == "auto":
            t_x = puller.autotune_exchange()
            log(rank, "exchange autotune (s over the first rounds): "
                + ", ".join(f"{m}={v:.3f}" for m, v in t_x.items()) + f" -> {puller.exchange}")
        else:
            puller.exchange = a.exchange

    def sync():
        if cuda:
            torch.cuda.synchronize()

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
            sync()
            puller.check()

    phase["autotune_s"] = round(time.time() - t_tune, 3)
    wd.arm("warmup")
    t_warm = time.time()
    try:
        warmup()
    except ops.IngestError as e:  # the error word is all-reduced: every rank takes this branch
        # (gloo moves device tensors only through its collectives -- a batched isend/irecv of device
        # tensors never completes -- so a gloo rehearsal falls back to its broadcasts)
        safe = "bcast" if (cuda and dist is not None and dist.get_backend() == "gloo") else "p2p"
        if world_size == 1 or puller.exchange == safe:  # the fallback itself failed
            raise
        log(rank, f"exchange {puller.exchange} failed verification ({e}); falling back to {safe}")
        puller.exchange = safe
        warmup()
    phase["warmup_s"] = round(time.time() - t_warm, 3)
    puller.err.zero_()
    wd.arm("timed")
    barrier()
    sync()
    hw0 = dict(puller.xchg.host_wait_s)
    t0, c0, thr0 = time.perf_counter(), time.process_time(), _thread_cpu()
    for _ in range(a.steps):
        puller.step()
    sync()
    barrier()
    t1 = time.perf_counter()
    phase["timed_cpu_s"] = round(time.process_time() - c0, 3)  # this rank's CPU seconds over the timed steps
    phase["timed_thread_cpu_s"] = _thread_cpu_delta(thr0, _thread_cpu(), top=6)
    wd.arm("report")
    puller.check()  # all timed steps verified (first error persists)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    recv = torch.tensor([float(puller.bytes_received)], dtype=torch.float64, device=device)
    ing = torch.tensor([float(puller.bytes_ingested)], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(recv)
        dist.all_reduce(ing)
    step_s = float(elapsed.item()) / max(1, a.steps)
    phase["timed_s"] = round(float(elapsed.item()), 3)
    # what each rank received from its peers per step, over the measured step time (GB/s)
    rx = [float(puller.bytes_received) / step_s / 1e9]
    if dist is not None:
        rx_all = [None] * world_size
        dist.all_gather_object(rx_all, rx[0])
        rx = rx_all
    res = {
        "mode": mode, "step_s": step_s, "model_bytes": world.model_bytes,
        "value": world_size * world.model_bytes / step_s / 1e9,
        "p2p_ratio": float(recv.item()) / (world_size * world.model_bytes),
        "ingest_GBps": float(ing.item()) / step_s / 1e9,
        "stored_ratio": float(world.chunk_clen.sum()) / float(world.chunk_len.sum()),
        "files": len(world.xet_files), "chunks": world.n_chunks, "xorbs": world.n_xorbs,
        "terms": int(len(world.terms)), "rounds": puller.n_rounds,
        "exchange": puller.exchange if world_size > 1 else "none",
        "exchange_autotune_s": {m: round(v, 4) for m, v in puller.exchange_times.items()},
        "hip_graph": bool(graph), "pipeline": getattr(puller, "pipeline", "cpu"), "seeders": seeders,
        "phase_s": phase, "exchange_rx_GBps": [round(x, 6) for x in rx],
    }
    if world_size > 1 and puller.exchange in ("ipc", "xgmi"):
        # host time per timed step in the peer-mapped issue path's ready-event waits + host barriers
        # (rank 0; the GPU keeps running the next round's copy and kernels meanwhile)
        hw = puller.xchg.host_wait_s
        # True: the exchanges waited on the GPU for the owners' ready counters (no host waits)
        res["ipc_signals"] = bool(puller.xchg.signaled)
        res["ipc_host_wait_ms_per_step"] = {
            k: round((hw[k] - hw0[k]) * (1e3 if k != "calls" else 1) / max(1, a.steps), 3) for k in hw}
    if keep is not None:  # the swarm row serves its CDN from this world's pinned origin
        keep["world"], keep["puller"] = world, puller
        return res
    puller.close()
    del puller, arena
    return res


def run_swarm_row(a, keep, device, rank, world_size, dist, wd, arenas=None) -> dict:
    """Time the public path on the world the engine just pulled: zest_amd.parallel.swarm_pull (what
    zest_amd.pull(repo, device="all") runs), listing + reconstructions from an in-process fake hub,
    every term's CDN fetch served from this rank's pinned origin through a mem:// memory CAS (the
    same cache -> P2P -> CDN waterfall, the bytes copied into the pinned staging like a NIC's DMA),
    then DeviceXetPull's pipeline (copy stream H2D || GPU decode + BLAKE3), the exchange at N > 1 and
    the Merkle check of every file.  A step is one whole swarm_pull call; the fetch pipelines and
    the arena (peer-mapped at N > 1) are kept between calls (reuse_pipeline, reuse_arena: each call's
    tensors are dropped before the next; the arena is the engine's, poisoned before the warm-up
    call, so the row's exchange is verified against bytes no earlier pull wrote), reconstructions
    are asked for anew every call.  The xorb
    cache is empty and cache writes are off (a device pull into HBM; nothing is read from disk)."""
    import tempfile

    import numpy as np
    import torch

    import importlib

    from zest_amd import ops
    from zest_amd.testing import FakeHub
    sp = importlib.import_module("zest_amd.parallel.swarm_pull")  # the module (the package re-exports the function)

    world, puller = keep["world"], keep["puller"]
    cuda = device.type == "cuda"
    wd.arm("swarm_setup")
    t_setup = time.time()
    # The engine's device buffers go first (its staging and tables; the row's pipelines allocate
    # their own).  The row's pulls land in the engine's arena: freeing 141 GB and allocating it again
    # costs the driver's reclaim, and a peer-imported VMM arena is not returned before every importing
    # process exits (profiles/r6/vmm_release_r6h_r6i/), so a fresh one would not fit next to it.  The
    # arena -- and the peers' mappings of it, which the next mode's engine exchanges through -- stay in
    # `arenas`.  The arena is poisoned first, on every rank before the barrier below, so the row's
    # first exchange is verified against bytes no earlier pull wrote.
    free0 = torch.cuda.mem_get_info(device)[0] if cuda else 0
    puller.release_device()
    arena = (arenas or {}).get("arena")
    if arena is not None:
        if cuda:
            arena.fill_(0xA5)
            torch.cuda.synchronize()
        sp.adopt_arena(arena)
    del arena
    import gc
    gc.collect()
    if cuda:
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    free1 = torch.cuda.mem_get_info(device)[0] if cuda else 0
    if dist is not None and world_size > 1:
        # every rank has released the engine's device buffers before any rank allocates the row's
        # pipelines (the 8-rank one-GPU rehearsal shares one card's memory between the ranks:
        # profiles/r5/rehearsal_n8_r5am.log ran out of it without this barrier)
        dist.barrier()
        if cuda:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    if cuda:
        # The driver reclaims (clears) freed device memory asynchronously, ~35 GB/s
        # (profiles/r5/alloc_probe_141g_r5aj.log): the engine's 141 GB arena is still counted as used
        # for seconds after its last reference went, and an allocation in that window can fail
        # instead of waiting (the 8-rank one-GPU rehearsal: hipMalloc out of memory with every VMM
        # mapping already released).  Wait until the free device memory stops growing.
        _wait_device_reclaim(device)
    if cuda:  # (device memory free before / after the engine's buffers were released, and after the barrier)
        own, imp = ops.hip().vmm_live()
        log(rank, f"[swarm_pull] device free GB: {free0 / 1e9:.1f} -> {free1 / 1e9:.1f} -> "
                  f"{torch.cuda.mem_get_info(device)[0] / 1e9:.1f}; live VMM mappings: own {own / 1e9:.1f} GB, "
                  f"imported {imp / 1e9:.1f} GB")
    hub = FakeHub()
    hub.xorb_url = "mem://origin"
    hub.start()
    hub.add_world(world, exact=True, payload=False)
    T = world.terms
    a_r, b_r = puller.rank_terms[rank]
    ts = range(a_r, b_r)
    ops.mem_origin_clear()
    ops.mem_origin_add([world.xorb_hash_hex(int(T["xorb"][t])) for t in ts], [int(T["ser0"][t]) for t in ts],
                       [puller.origin.ptr + int(puller.term_origin_off[t - a_r]) for t in ts],
                       [int(T["ser_len"][t]) for t in ts])
    cache = tempfile.mkdtemp(prefix="zest-bench-cache-")
    for k, v in hub.env(cache).items():
        os.environ[k] = v
    os.environ["ZEST_CACHE_WRITES"] = "0"
    # timed HIP events around every staging batch's H2D copy and kernels: the row reports how much of
    # the copy time ran under the decode/hash kernels (DeviceXetPull.timeline_json)
    os.environ.setdefault("ZEST_DEVICE_TIMING", "1")
    own_pg = False
    if dist is None:  # one rank: swarm_pull is a collective over a group of one
        import torch.distributed as tdist
        tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
        own_pg = True
    import torch.distributed as tdist
    if world_size > 1 and rank == 0:
        _log_split_check(world, puller, world_size, sp)
    setup_s = time.time() - t_setup

    def one(st):
        out = sp.swarm_pull(world.spec.repo_id, device=device if cuda else None, p2p=False, dht=False,
                            round_bytes=a.round_mb << 20, stats=st, reuse_pipeline=True, reuse_arena=True)
        n = len(out)
        del out
        return n

    wd.arm("swarm_warmup")
    t_w = time.time()
    warm_st: dict = {}
    for i in range(a.swarm_warmup):
        one(warm_st if i == 0 else {})  # the first call's phases: what a user's first pull costs
    warm_s = time.time() - t_w
    wd.arm("swarm_timed")
    from zest_amd import _core
    _core.trace.roctx_push("swarm_pull timed")  # (ZEST_ROCTX=1: the window of tools/gpu/overlap.py --marker)
    mark = cuda and os.environ.get("ZEST_BENCH_MARK") == "1"
    if mark:  # a distinctive kernel brackets the timed window in a kernel trace (overlap.py --between)
        torch.cuda._sleep(1000)
    times, st, step_phases = [], {}, []
    thr0 = _thread_cpu()
    ctx0 = {k[0]: _thread_ctx(k[0]) for k in thr0}
    sampler = _SyscallSampler() if os.environ.get("ZEST_BENCH_SPIN_PROBE") == "1" else None
    prof = None
    if os.environ.get("ZEST_BENCH_PYPROF") == "1":  # Python profile of the timed calls (pulling thread)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    for _ in range(a.swarm_steps):
        st = {}
        tdist.barrier()
        if cuda:
            torch.cuda.synchronize()
        t0, c0 = time.perf_counter(), time.process_time()
        n_t = one(st)
        if cuda:
            torch.cuda.synchronize()
        t_pull = time.perf_counter() - t0
        cpu = time.process_time() - c0  # CPU seconds of every thread of this rank during the call
        tdist.barrier()
        times.append(time.perf_counter() - t0)
        # every timed step's phases on this rank (a slow step is then attributable to a phase and
        # a rank: VERDICT r5 weak 2); "other_s" = the call's wall time outside the named phases
        ph = {k: v for k, v in (st.get("phases") or {}).items() if k == "plan_s" or not k.startswith("plan_")}
        named = sum(v for k, v in ph.items() if k in ("init_s", "plan_s", "possession_s", "alloc_s", "shard_s",
                                                       "setup_exchange_s", "pull_s", "verify_s", "repair_s",
                                                       "tensors_s"))
        step_phases.append(ph | {"call_s": round(t_pull, 4), "other_s": round(t_pull - named, 4), "cpu_s": round(cpu, 4),
                                 "item_ready_s": st.get("item_ready_s", []),
                                 "timeline": st.get("device_timeline", {})})
    thr1 = _thread_cpu()
    thr = _thread_cpu_delta(thr0, thr1)  # where this rank's CPU went over the timed calls
    busiest = _busiest_threads(thr0, thr1, ctx0)
    if sampler is not None and busiest:
        busiest[0].append(sampler.report(busiest[0][1]))  # what the busiest thread was doing
    if prof is not None:
        import io
        import pstats
        prof.disable()
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(25)
        log(rank, f"[swarm_pull] Python profile of the timed calls (pulling thread):\n{buf.getvalue()}")
    if mark:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    _core.trace.roctx_pop()
    dev_t = device if (cuda and not own_pg) else "cpu"
    el = torch.tensor(times, dtype=torch.float64, device=dev_t)
    rx = torch.tensor([float(st.get("received_bytes", 0))], dtype=torch.float64, device=dev_t)
    if world_size > 1:
        tdist.all_reduce(el, op=tdist.ReduceOp.MAX)  # every step at its slowest rank
        tdist.all_reduce(rx)
    wd.arm("swarm_report")
    log(rank, f"[swarm_pull] world {st.get('world')} fetched {st.get('fetched_bytes')} received "
              f"{st.get('received_bytes')} items {st.get('items')} rounds {st.get('rounds')} exchange {st.get('exchange')}")
    times = el.cpu().tolist()
    step_s = float(sum(times) / len(times))
    all_phases, all_thr, all_busy = [step_phases], [thr], [busiest]
    if world_size > 1:
        all_phases = [None] * world_size
        tdist.all_gather_object(all_phases, step_phases)
        all_thr = [None] * world_size
        tdist.all_gather_object(all_thr, thr)
        all_busy = [None] * world_size
        tdist.all_gather_object(all_busy, busiest)
    # agree_s is this rank's wait at the end of a streamed pull for the last rounds' gathers: the
    # time until the slowest rank queued its last item (skew) plus the agreement's own cost.  Per
    # timed step: the largest own cost over the ranks (agree_s - skew), as a fraction of pull_s.
    own = []
    try:
        for k in range(len(all_phases[0])):
            last = [ph[k]["item_ready_s"][-1] for ph in all_phases if ph[k].get("item_ready_s")]
            if len(last) != len(all_phases):
                break
            mx = max(last)
            own.append(max((ph[k].get("agree_s", 0.0) - (mx - ph[k]["item_ready_s"][-1])) / max(1e-9, ph[k].get("pull_s", 0.0))
                           for ph in all_phases))
    except (KeyError, IndexError, TypeError):
        own = []
    sp.release_pipelines()
    ops.mem_origin_clear()
    hub.stop()
    if own_pg:
        tdist.destroy_process_group()
    total = st.get("total_bytes", world.model_bytes)
    return {"swarm_pull_GBps": round(world_size * total / step_s / 1e9, 3),
            "swarm_pull_ms_per_step": round(step_s * 1e3, 3),
            "swarm_pull_step_s": [round(x, 4) for x in times],
            "swarm_pull_mode": keep.get("mode"), "swarm_pull_tensors": n_t,
            "swarm_pull_p2p_ratio": round(float(rx.item()) / (world_size * total), 4) if total else 0.0,
            "swarm_pull_exchange": st.get("exchange"), "swarm_pull_phases": st.get("phases"),
            "swarm_pull_streamed": st.get("streamed"),
            # [rank][timed step] -> phases of that call on that rank
            "swarm_pull_step_phases": all_phases,
            "swarm_pull_agree_own_frac": [round(x, 4) for x in own],
            # [rank] -> CPU seconds per thread name over the timed calls
            "swarm_pull_thread_cpu_s": all_thr,
            # [rank] -> the busiest threads: [name, tid, cpu_s, voluntary, involuntary switches]
            "swarm_pull_busiest_threads": all_busy,
            "swarm_pull_fetch": {k: st.get("fetch_stats", {}).get(k) for k in ("bytes_from_cdn", "bytes_from_cache",
                                                                                  "bytes_from_peer")},
            "swarm_pull_device_timeline": st.get("device_timeline"),
            "swarm_pull_setup_s": round(setup_s, 3), "swarm_pull_warmup_s": round(warm_s, 3),
            "swarm_pull_first_call_phases": warm_st.get("phases", {}), "swarm_pull_first_call_alloc": warm_st.get("alloc", {}),
            "swarm_pull_arena_reused": bool(st.get("alloc", {}).get("reused", False)),
            "swarm_pull_rank_terms": [a_r, b_r], "swarm_pull_n_origin_runs": len(ts),
            "swarm_pull_verify": "merkle file hashes of every file on every rank"}


def _thread_cpu() -> dict:
    """CPU seconds (user + system) of every thread of this process, by (tid, name) -- Linux /proc."""
    out = {}
    tick = os.sysconf("SC_CLK_TCK")
    try:
        tids = os.listdir("/proc/self/task")
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"/proc/self/task/{tid}/comm") as fh:
                comm = fh.read().strip()
            with open(f"/proc/self/task/{tid}/stat") as fh:
                st = fh.read()
            f = st[st.rindex(")") + 2:].split()
            out[(tid, comm)] = (int(f[11]) + int(f[12])) / tick
        except (OSError, ValueError, IndexError):
            continue
    return out


def _thread_ctx(tid: str) -> tuple[int, int]:
    """(voluntary, involuntary) context switches of a thread of this process."""
    v = n = 0
    try:
        with open(f"/proc/self/task/{tid}/status") as fh:
            for ln in fh:
                if ln.startswith("voluntary_ctxt_switches"):
                    v = int(ln.split()[1])
                elif ln.startswith("nonvoluntary_ctxt_switches"):
                    n = int(ln.split()[1])
    except (OSError, ValueError):
        pass
    return v, n


def _busiest_threads(a: dict, b: dict, ctx0: dict, top: int = 6) -> list:
    """The `top` threads by CPU seconds between two _thread_cpu() snapshots: [name, tid, cpu_s,
    voluntary switches, involuntary switches] -- a thread that polls shows CPU with few voluntary
    switches."""
    rows = []
    for k, v in b.items():
        d = v - a.get(k, 0.0)
        if d > 0:
            c1 = _thread_ctx(k[0])
            c0 = ctx0.get(k[0], (0, 0))
            rows.append([k[1], int(k[0]), round(d, 3), c1[0] - c0[0], c1[1] - c0[1]])
    rows.sort(key=lambda r: -r[2])
    return rows[:top]


class _SyscallSampler:
    """ZEST_BENCH_SPIN_PROBE=1: samples /proc/self/task/*/syscall every 20 ms on a thread of its own
    and reports, for a given thread, how often it was in user space ("running") or in which system
    call, and the libraries its system calls were made from (their pc against /proc/self/maps)."""

    def __init__(self):
        import collections
        self.hist = collections.defaultdict(collections.Counter)
        self.libs = collections.defaultdict(collections.Counter)
        self.stop = threading.Event()
        self.maps = []
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def _lib(self, pc: int) -> str:
        if not self.maps:
            try:
                with open("/proc/self/maps") as fh:
                    for ln in fh:
                        f = ln.split()
                        lo, hi = (int(x, 16) for x in f[0].split("-"))
                        self.maps.append((lo, hi, f[5] if len(f) > 5 else "?"))
            except OSError:
                return "?"
        for lo, hi, name in self.maps:
            if lo <= pc < hi:
                return os.path.basename(name)
        return "?"

    def _caller(self, sp: int) -> str:
        """The first return address on the thread's stack (near sp) that lies outside libc: the
        library that made the system call (a heuristic scan of 64 words)."""
        import ctypes
        import struct
        try:
            words = struct.unpack("<64Q", ctypes.string_at(sp, 512))
        except (OSError, ValueError, struct.error):
            return "?"
        for w in words:
            lib = self._lib(w)
            if lib not in ("?", "libc.so.6", "[stack]", "[heap]", "") and not lib.startswith("["):
                return lib
        return "libc.so.6"

    def _run(self):
        while not self.stop.wait(0.02):
            try:
                tids = os.listdir("/proc/self/task")
            except OSError:
                continue
            for tid in tids:
                try:
                    with open(f"/proc/self/task/{tid}/syscall") as fh:
                        f = fh.read().split()
                except OSError:
                    continue
                if not f:
                    continue
                self.hist[int(tid)][f[0]] += 1
                if f[0] not in ("running", "-1") and len(f) >= 9:
                    try:
                        self.libs[int(tid)][self._caller(int(f[7], 16))] += 1
                    except ValueError:
                        pass

    def report(self, tid: int) -> dict:
        self.stop.set()
        self.th.join(1.0)
        return {"states": dict(self.hist[tid].most_common(6)), "libs": dict(self.libs[tid].most_common(4))}


def _thread_cpu_delta(a: dict, b: dict, top: int = 10) -> dict:
    """CPU seconds per thread name between two _thread_cpu() snapshots (the largest `top`)."""
    by: dict = {}
    for k, v in b.items():
        by[k[1]] = by.get(k[1], 0.0) + v - a.get(k, 0.0)
    return {k: round(v, 3) for k, v in sorted(by.items(), key=lambda kv: -kv[1])[:top] if v > 0}


def _wait_device_reclaim(device, timeout_s: float = 30.0, quiet_s: float = 0.5) -> float:
    """Poll the device's free memory until it has not grown for `quiet_s` (or `timeout_s` passed);
    returns the seconds waited."""
    import torch
    t0 = time.time()
    last, since = torch.cuda.mem_get_info(device)[0], time.time()
    while time.time() - t0 < timeout_s:
        time.sleep(0.05)
        free = torch.cuda.mem_get_info(device)[0]
        if free > last:
            last, since = free, time.time()
        elif time.time() - since >= quiet_s:
            break
    return time.time() - t0


def _log_split_check(world, puller, world_size, sp) -> None:
    """Diagnostics (rank 0, N > 1): the public path's term owners -- computed the way swarm_pull will,
    on the files in the order the hub lists them -- against the engine's per-rank origin shares that
    each rank's memory CAS serves.  A term owned by a rank whose origin lacks it is a 404 in the row."""
    import numpy as np

    from zest_amd import _core
    try:
        _, files = _core.list_repo_files(world.spec.repo_id, "main", "model")
        by_hash = {world.file_hash_hex(i): i for i in range(len(world.xet_files))}
        order = [by_hash[f["xet_hash"]] for f in files if f["path"].endswith(".safetensors") and f["xet_hash"]]
        T = world.terms
        idx = np.concatenate([np.flatnonzero(T["file"] == i) for i in order]) if order else np.zeros(0, np.int64)
        owner = sp.assign_owners(T["ulen"][idx], None, world_size)
        rt = puller.rank_terms
        eng = np.empty(len(T), dtype=np.int64)
        for r, (a, b) in enumerate(rt):
            eng[a:b] = r
        bad = np.flatnonzero(eng[idx] != owner)
        log(0, f"[swarm_pull] split check: {len(idx)} of {len(T)} terms planned, files in listing order "
               f"{order[:8]}{'...' if len(order) > 8 else ''}, engine shares {rt}; {len(bad)} terms owned "
               f"elsewhere" + (f" (first: plan term {int(bad[0])} = world term {int(idx[bad[0]])}, "
                               f"swarm rank {int(owner[bad[0]])}, engine rank {int(eng[idx[bad[0]]])})" if len(bad) else ""))
    except Exception as e:  # noqa: BLE001 - diagnostics only
        log(0, f"[swarm_pull] split check failed: {type(e).__name__}: {e}")


def _headline(a, spec, results, world_size, cuda, backend, rccl_ranks, devices, distinct, numa_cpus) -> dict:
    """The JSON line of the modes measured so far (the first mode is the headline `value`)."""
    head = results[0]
    seeders = head["seeders"]
    out = {
        "metric": metric_name(spec),
        "value": round(head["value"], 3),
        "unit": "GB/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(head["step_s"] * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": _data_note(head) + ("" if cuda else "; CPU gloo rehearsal, not a GPU measurement"),
        "p2p_ratio": round(head["p2p_ratio"], 4),
        "ingest_GBps": round(head["ingest_GBps"], 3),
        "extra": {f"{r['mode']}_GBps": round(r["value"], 3) for r in results}
        | {f"{r['mode']}_ms_per_step": round(r["step_s"] * 1e3, 3) for r in results}
        | {f"{r['mode']}_p2p_ratio": round(r["p2p_ratio"], 4) for r in results}
        | {f"{r['mode']}_stored_ratio": round(r["stored_ratio"], 4) for r in results},
        "config": {"model": spec.repo_id, "global_batch": world_size, "seq_len": None,
                   "parallelism": (f"swarm{world_size}" if seeders == world_size
                                   else f"seed{seeders}-leech{world_size - seeders}"),
                   "data_mode": head["mode"], "modes": [r["mode"] for r in results],
                   "model_bytes": head["model_bytes"], "files": head["files"],
                   "chunks": head["chunks"], "xorbs": head["xorbs"], "terms": head["terms"],
                   "rounds": head["rounds"], "round_mb": a.round_mb, "exchange": head["exchange"],
                   "exchange_autotune_s": head["exchange_autotune_s"],
                   "verify": "blake3 of every chunk on every rank + merkle file hashes",
                   "numa_bound_cpus": len(numa_cpus), "hip_graph": head["hip_graph"],
                   "pipeline": head["pipeline"], "device": a.device,
                   "backend": backend if world_size > 1 else "none",
                   "rccl_ranks": rccl_ranks, "devices": devices, "distinct_devices": distinct,
                   "phase_s": head["phase_s"], "exchange_rx_GBps": head["exchange_rx_GBps"]},
    }
    if "ipc_host_wait_ms_per_step" in head:
        out["extra"]["ipc_host_wait_ms_per_step"] = head["ipc_host_wait_ms_per_step"]
        out["extra"]["ipc_signals"] = head.get("ipc_signals", False)
    return out


def _swarm_extra(rows: dict, results: list) -> dict:
    """extra fields of the public-path rows: the first mode's row under the plain swarm_pull_* keys,
    every mode's throughput under swarm_pull_<mode>_* with its ratio to the engine on the same world."""
    if not rows:
        return {}
    first = next(iter(rows))
    ex = dict(rows[first])
    engine = {r["mode"]: r["value"] for r in results}
    by_mode = {}
    for mode, row in rows.items():
        if "swarm_pull_GBps" not in row:
            ex[f"swarm_pull_{mode}_error"] = row.get("swarm_pull_error")
            continue
        ex[f"swarm_pull_{mode}_GBps"] = row["swarm_pull_GBps"]
        ex[f"swarm_pull_{mode}_ms_per_step"] = row["swarm_pull_ms_per_step"]
        ex[f"swarm_pull_{mode}_vs_engine"] = round(row["swarm_pull_GBps"] / engine[mode], 4) if engine.get(mode) else None
        by_mode[mode] = {k: row.get(f"swarm_pull_{k}") for k in ("GBps", "ms_per_step", "step_s", "streamed", "exchange",
                                                                  "p2p_ratio", "phases", "first_call_phases")}
    ex["swarm_pull_modes"] = by_mode
    return ex


def _data_note(r: dict) -> str:
    what = "N(0,0.02) bf16 weights" if r["mode"] == "bf16" else "uniformly random bytes"
    if r["stored_ratio"] < 1.0:
        stored = f"BG4-LZ4 compressed chunks as Xet stores bf16 checkpoints, stored/raw {r['stored_ratio']:.3f}"
    else:
        stored = "chunks stored raw"
    return (f"synthetic ({what} of the real tensor shapes; real Xet CDC/xorbs/hashes; {stored}; "
            "origin = pinned host memory standing in for the CDN)")


def device_id(device) -> str:
    """PCI address of a GPU ("cpu" for host rehearsals)."""
    import torch
    if device.type != "cuda":
        return "cpu"
    p = torch.cuda.get_device_properties(device)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"


def topology(dist, device, world_size: int):
    """(ranks the collective backend counted, every rank's device PCI address, all distinct?).  The
    count is an all_reduce of ones on the job's default group (RCCL on GPUs): proof of how many
    ranks the measured collectives really spanned."""
    import torch
    me = device_id(device)
    if dist is None:
        return 1, [me], me != "cpu"
    one = torch.ones(1, dtype=torch.int32, device=device)
    dist.all_reduce(one)
    ids = [None] * world_size
    dist.all_gather_object(ids, me)
    return int(one.item()), ids, len(set(ids)) == world_size and "cpu" not in ids


# HIP hardware queues per process (GPU_MAX_HW_QUEUES; HIP's default, and the box's setting, is 4).
# A rank drives up to ~9 streams (copy, two compute lanes, verify, up to four peer-copy streams or
# the all-gather unpack, the caller's) and HIP maps streams onto the hardware queues round-robin, so
# with 4 queues independent streams share in-order queues.  8 measured neutral at N = 1 (70B:
# 64.44 / 56.85 GB/s vs 64.23 / 56.83 with 4, profiles/r4/bench_hwq8_r4g.log).  Set before HIP starts.
HW_QUEUES = "8"


def rank_main(a) -> None:
    # Only when every rank has a GPU of its own: ranks sharing one GPU (the gloo rehearsal) would
    # stack 4 x 8 queues on one device, and the 4-rank rehearsal ran 133-150 GB/s with 8 queues per
    # rank against 186 with 4 (profiles/r4/rehearsal_r4d.log, rehearsal_n4_hwq8_r4l.log).
    if (a.device == "cuda" and (os.environ.get("ZEST_BENCH_BACKEND", "nccl") == "nccl"
                                or os.environ.get("ZEST_BENCH_HW_QUEUES")) and os.environ.get("ZEST_BENCH_HW_QUEUES", HW_QUEUES) != "0"):
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZEST_BENCH_HW_QUEUES", HW_QUEUES)
    import torch

    from zest_amd import models, ops

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != a.gpus:
        log(rank, f"--gpus {a.gpus} but WORLD_SIZE={world_size}: running {world_size} ranks")
    wd = Watchdog(rank, world_size > 1)
    wd.arm("init")
    # ZEST_BENCH_BACKEND=gloo is a rehearsal mode for one-GPU boxes: several ranks share the device,
    # control traffic goes over gloo.  Its numbers are not xGMI measurements; config.backend says so.
    cuda = a.device == "cuda"
    backend = os.environ.get("ZEST_BENCH_BACKEND", "nccl" if cuda else "gloo")
    if cuda:
        n_dev = max(1, torch.cuda.device_count())
        device = torch.device("cuda", local_rank % n_dev if backend == "gloo" else local_rank)
        torch.cuda.set_device(device)
        from zest_amd.parallel import bind_local_numa
        numa_cpus = bind_local_numa(device)
        if numa_cpus:
            log(rank, f"bound to {len(numa_cpus)} CPUs on the GPU's NUMA node")
        ops.hip()
    else:
        device, numa_cpus = torch.device("cpu"), []
    dist = None
    if world_size > 1:
        import datetime

        import torch.distributed as dist
        timeout = datetime.timedelta(seconds=float(os.environ.get("ZEST_BENCH_PG_TIMEOUT", "300")))
        if backend == "gloo":
            dist.init_process_group("gloo", timeout=timeout)
        else:
            from zest_amd.parallel import nccl_options
            dist.init_process_group("nccl", device_id=device, pg_options=nccl_options(), timeout=timeout)
    rccl_ranks, devices, distinct = topology(dist, device, world_size)
    log(rank, f"collective ranks {rccl_ranks} ({backend if dist is not None else 'none'}), devices {devices}")
    if backend == "nccl" and dist is not None and (not distinct or rccl_ranks != world_size):
        # an RCCL number only counts when every rank drove its own GPU
        raise SystemExit(f"refusing an nccl run over {devices} ({rccl_ranks} ranks counted by the collective)")
    spec = models.get(a.model)
    results, pick, arenas = [], None, {}
    # (CPU rehearsals run it only when asked: --swarm-row on)
    swarm_row = ((a.swarm_row == "auto" and cuda) or a.swarm_row == "on") and a.seeders in (0, world_size)
    swarm_rows: dict = {}  # mode -> the public-path row measured on that mode's world
    out: dict = {}
    printed = [False]

    def emit(extra_fields: dict) -> None:  # the one JSON line, printed once by rank 0
        if rank == 0 and not printed[0] and out:
            printed[0] = True
            print(json.dumps(out | {"extra": out["extra"] | extra_fields}), flush=True)

    for i, mode in enumerate(a.modes):
        keep = {} if swarm_row else None
        r = run_mode(a, mode, spec, device, rank, world_size, dist, wd, exchange_pick=pick, arenas=arenas,
                     keep=keep)
        pick = r["exchange"] if world_size > 1 else None
        log(rank, f"[{mode}] {r['value']:.3f} GB/s aggregate, {r['step_s'] * 1e3:.1f} ms/step, "
                  f"exchange {r['exchange']}")
        results.append(r)
        out = _headline(a, spec, results, world_size, cuda, backend, rccl_ranks, devices, distinct, numa_cpus)
        if keep:
            # The public-path row runs on every data mode's world, right after the engine measured it
            # (its CDN is served from that world's pinned origin).  At N > 1 it must not cost the
            # headline: an exception is recorded in extra.swarm_pull_error, and a phase that overruns its
            # deadline prints the headline line (the modes measured so far) with the row marked failed
            # and exits 0 (Watchdog.fallback).
            keep["mode"] = mode
            if world_size > 1:
                wd.fallback = lambda reason: emit(_swarm_extra(swarm_rows, results) | {"swarm_pull_error": reason})
            try:
                swarm_rows[mode] = run_swarm_row(a, keep, device, rank, world_size, dist, wd, arenas)
                log(rank, f"[swarm_pull {mode}] {swarm_rows[mode]['swarm_pull_GBps']:.3f} GB/s aggregate, "
                          f"{swarm_rows[mode]['swarm_pull_ms_per_step']:.1f} ms/step (public path, memory CAS)")
            except Exception as e:  # noqa: BLE001 - the headline stands without the row
                if world_size == 1:
                    raise
                swarm_rows[mode] = {"swarm_pull_error": f"{type(e).__name__}: {e}"[:1000]}
                log(rank, f"[swarm_pull {mode}] failed: {swarm_rows[mode]['swarm_pull_error']}")
            keep["puller"].close()
            keep.clear()
            wd.fallback = None
    if swarm_row:
        wd.arm("report")
    emit(_swarm_extra(swarm_rows, results))
    # (the pinned origin pool is left to the process exit: unregistering ~141 GB one buffer at a time
    # only delays it)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    wd.disarm()


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        t = os.environ.get("ZEST_BENCH_TIMEOUT")
        return launch_ranks(a.gpus, argv, float(t) if t else None)
    rank_main(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
