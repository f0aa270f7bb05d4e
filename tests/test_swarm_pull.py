"""Intra-node swarm pull (zest_amd.parallel.swarm_pull) over gloo process groups on CPU: every rank
ends with every tensor, each Xet file fetched from the (fake) hub by exactly one owner rank, the rest
received from peers and re-verified; a rank whose fetch fails makes every rank raise (no hang).
The GPU variant (device-direct fetch + RCCL/gloo broadcast of device buffers) is in
test_gpu_device.py."""
from __future__ import annotations

import dataclasses
import json
import os
import struct

import pytest
import torch
import torch.multiprocessing as mp

from e2e_util import free_port
from zest_amd import models
from zest_amd.synthetic import SyntheticWorld
from zest_amd.testing import FakeHub


def _sharded_world(seed: int) -> SyntheticWorld:
    spec = dataclasses.replace(models.get("llama-tiny"), max_shard_bytes=700_000)
    return SyntheticWorld(spec, seed=seed, mode="bf16")


def _expected(world):
    out = {}
    for f in world.xet_files:
        data = world.file_bytes_host(f)
        (hlen,) = struct.unpack("<Q", data[:8])
        for name, ent in json.loads(data[8:8 + hlen]).items():
            if name != "__metadata__":
                a, b = ent["data_offsets"]
                out[name] = data[8 + hlen + a:8 + hlen + b]
    return out


def _worker(rank, world_size, port, repo, q, peers=None):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from zest_amd.parallel import swarm_pull
        st = {}
        try:
            t = swarm_pull(repo, p2p=bool(peers), peers=peers, dht=False, stats=st)
            q.put((rank, "ok", {k: v.contiguous().view(torch.uint8).numpy().tobytes() for k, v in t.items()}, st))
        except Exception as e:
            q.put((rank, type(e).__name__, str(e), st))
    finally:
        dist.destroy_process_group()


def _run(world_size, repo, peers=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, repo, q, peers)) for r in range(world_size)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.fixture
def hub_env(tmp_path, monkeypatch):
    world = _sharded_world(21)
    assert len(world.xet_files) >= 3  # several owners
    hub = FakeHub(policy="auto", max_xorb_bytes=256 << 10)
    hub.start()
    hub.add_world(world)
    for k, v in hub.env(str(tmp_path)).items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
    yield world, hub
    hub.stop()


@pytest.mark.parametrize("world_size", [1, 3])
def test_swarm_pull_every_rank_gets_every_tensor(hub_env, world_size):
    world, hub = hub_env
    want = _expected(world)
    res = _run(world_size, world.spec.repo_id)
    assert [r[1] for r in res] == ["ok"] * world_size, res
    for _, _, got, _ in res:
        assert got.keys() == want.keys()
        assert all(got[k] == want[k] for k in want)
    # each file crossed the network once: owners' fetched bytes add up to the model, and each rank
    # received exactly what it did not fetch
    total = sum(f.size for f in world.xet_files)
    assert sum(r[3]["fetched_bytes"] for r in res) == total
    for r in res:
        assert r[3]["fetched_bytes"] + r[3]["received_bytes"] == total
    assert hub.counters.get("xorb_get", 0) > 0


@pytest.mark.parametrize("victim_index", [0, -1])
def test_swarm_pull_failed_owner_fails_every_rank(hub_env, victim_index):
    world, hub = hub_env
    # the CDN refuses every xorb behind one file: its owner cannot fetch it (file 0: a first-round
    # fetch; the last file: a later round, after earlier rounds' broadcasts were issued)
    victim = world.xet_files[victim_index]
    xh = hub.xet_hash(world.spec.repo_id, victim.path)
    hub.fail_xorbs = {t["hash"] for t in hub.reconstruction(xh)["terms"]}
    res = _run(3, world.spec.repo_id)
    assert all(r[1] == "SwarmPullError" for r in res), res
    assert sum("rank" in r[2] for r in res) == 3


def test_swarm_pull_from_another_node(hub_env, tmp_path):
    """SURVEY §4.4 item 7, multi-node without a cluster: "node B" is a `zest serve` process with the
    model in its xorb cache; "node A" is 2 ranks running swarm_pull with B as their BEP XET peer over
    TCP loopback.  Every file crosses the inter-node link once (owner rank, 100 % from the peer, no
    CDN), is then broadcast inside node A, and every rank ends with every tensor."""
    from e2e_util import Node

    world, hub = hub_env
    b = Node(hub, tmp_path, "node_b")
    try:
        b.run("pull", world.spec.repo_id, "--no-p2p", "--no-serve", timeout=300)
        b.spawn("serve", "--listen-port", str(b.listen_port), "--http-port", str(b.http_port))
        b.wait_healthy()
        want = _expected(world)
        before = hub.counters.get("xorb_get", 0)
        res = _run(2, world.spec.repo_id, peers=[f"127.0.0.1:{b.listen_port}"])
        assert [r[1] for r in res] == ["ok", "ok"], res
        for _, _, got, _ in res:
            assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert hub.counters.get("xorb_get", 0) == before, "node A touched the CDN"
        total = sum(f.size for f in world.xet_files)
        assert sum(r[3]["fetched_bytes"] for r in res) == total
        st = __import__("json").loads(b.api("/v1/status")[1])
        assert st["bytes_served"] > 0
    finally:
        b.close()


def _api_worker(rank, world_size, port, repo, q, fault):
    """zest_amd.pull(repo, device="all") on a CPU process group (gloo)."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fault:
        os.environ["ZEST_SWARM_FAULT"] = fault
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        import zest_amd
        from zest_amd.parallel import swarm_pull
        st = {}
        try:
            if fault:  # swarm_pull itself (the same call the public API makes)
                t = swarm_pull(repo, p2p=False, dht=False, stats=st)
            else:
                t = zest_amd.pull(repo, device="all", p2p=False, dht=False, stats=st)
            q.put((rank, "ok", {k: v.contiguous().view(torch.uint8).numpy().tobytes() for k, v in t.items()}, st))
        except Exception as e:
            q.put((rank, type(e).__name__, str(e), st))
    finally:
        dist.destroy_process_group()


def _run_api(world_size, repo, fault=""):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_api_worker, args=(r, world_size, port, repo, q, fault)) for r in range(world_size)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_pull_device_all_is_a_swarm_pull_without_snapshot(hub_env, tmp_path):
    """The public API's device="all" runs the swarm pull: every rank gets every tensor, each file
    is fetched once by its owner into memory, and no rank writes an HF snapshot."""
    world, hub = hub_env
    want = _expected(world)
    res = _run_api(3, world.spec.repo_id)
    assert [r[1] for r in res] == ["ok"] * 3, res
    for _, _, got, st in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert st["exchange"] in ("bcast", "allgather", "p2p") and st["world"] == 3  # the mode it used
    snaps = list((tmp_path / "hf").rglob("snapshots/*/*")) if (tmp_path / "hf").exists() else []
    assert not snaps, snaps


def test_swarm_pull_reshards_a_failed_fetch(hub_env):
    """Rank 1's first-round fetch fails (injected): its file is reassigned to another owner and
    every rank still ends with every tensor (SURVEY §5.3 re-shard), instead of all ranks raising."""
    world, hub = hub_env
    want = _expected(world)
    res = _run_api(3, world.spec.repo_id, fault="1:0")
    assert [r[1] for r in res] == ["ok"] * 3, res
    for _, _, got, _ in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
    assert all(r[3]["reassigned"] >= 1 for r in res)
    total = sum(f.size for f in world.xet_files)
    assert sum(r[3]["fetched_bytes"] for r in res) == total  # every file landed once


def _elastic_worker(rank, world_size, port, repo, q, fault, round_bytes):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZEST_SWARM_FAULT=fault,
                      ZEST_SWARM_CTL_TIMEOUT="20", ZEST_SWARM_HB_STALE="3")
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    from zest_amd.parallel import swarm_pull
    st = {}
    try:
        t = swarm_pull(repo, p2p=False, dht=False, stats=st, round_bytes=round_bytes)
        q.put((rank, "ok", {k: v.contiguous().view(torch.uint8).numpy().tobytes() for k, v in t.items()}, st))
    except Exception as e:
        q.put((rank, type(e).__name__, str(e), st))
    # no destroy_process_group: the default group still counts the dead rank


def _run_elastic(world_size, repo, fault, round_bytes, expect_dead=()):
    import queue as _q
    import time as _t
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_elastic_worker, args=(r, world_size, port, repo, q, fault, round_bytes))
             for r in range(world_size)]
    t0 = _t.monotonic()
    for p in procs:
        p.start()
    res = []
    for _ in range(world_size - len(expect_dead)):
        try:
            res.append(q.get(timeout=180))
        except _q.Empty:
            break
    dt = _t.monotonic() - t0
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    return sorted(res, key=lambda r: r[0]), [p.exitcode for p in procs], dt


def test_swarm_pull_round_synchronous_loop(hub_env, monkeypatch):
    """ZEST_SWARM_STREAM=0: the round-synchronous loop (agree, then exchange; two alternating
    pipelines) still pulls every tensor -- it is also what the streamed phase falls back to for
    reassigned ranges."""
    monkeypatch.setenv("ZEST_SWARM_STREAM", "0")
    world, hub = hub_env
    want = _expected(world)
    res, codes, _ = _run_elastic(3, world.spec.repo_id, "", 256 << 10)
    assert codes == [0, 0, 0] and [r[1] for r in res] == ["ok"] * 3, res
    for _, _, got, st in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert st["pipelined"] and not st["streamed"]


def test_swarm_pull_term_shards_and_stats(hub_env):
    """Ranks own byte-balanced *term* ranges (not whole files): each rank fetches ~1/3 of the model,
    in several rounds, and the stats say which exchange replicated them."""
    world, hub = hub_env
    want = _expected(world)
    total = sum(f.size for f in world.xet_files)
    res, codes, _ = _run_elastic(3, world.spec.repo_id, "", 256 << 10)
    assert codes == [0, 0, 0] and [r[1] for r in res] == ["ok"] * 3, res
    for _, _, got, st in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert st["exchange"] in ("bcast", "allgather", "p2p") and st["world"] == 3
        assert st["rounds"] >= 2 and st["items"] >= 6
        # streamed rounds (default): one persistent pipeline, exchanges issued before agreement
        assert st["streamed"] and not st["pipelined"]
        assert st["fetched_bytes"] + st["received_bytes"] == total
        assert abs(st["fetched_bytes"] - total / 3) < 0.2 * total, st["fetched_bytes"]
        assert set(st["phases"]) >= {"plan_s", "fetch_s", "agree_s", "verify_s", "pull_s"}


def test_swarm_pull_survives_a_lost_rank(hub_env):
    """SURVEY §5.3 elastic 3 -> 2: rank 2 dies (os._exit) at its second round.  Ranks 0 and 1 see the
    control collective fail, agree through the store that rank 2 is gone, rebuild their groups
    in-process and re-shard its unfinished ranges; both end with every tensor, verified, in bounded
    time."""
    world, hub = hub_env
    want = _expected(world)
    res, codes, dt = _run_elastic(3, world.spec.repo_id, "exit:2:1", 256 << 10, expect_dead=(2,))
    assert codes[2] == 1, codes
    assert [r[0] for r in res] == [0, 1] and [r[1] for r in res] == ["ok", "ok"], res
    for _, _, got, st in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert st["recovered_ranks"] == 1 and st["world"] == 2
    assert dt < 150, dt


def test_swarm_pull_eight_ranks_lose_two(hub_env):
    """N = 8 rehearsal on gloo: term shares over 8 ranks, then ranks 3 and 6 die in the same round;
    the six survivors agree on the member list once, re-shard both ranks' ranges and all finish
    with every tensor verified."""
    world, hub = hub_env
    want = _expected(world)
    res, codes, dt = _run_elastic(8, world.spec.repo_id, "exit:3:1,exit:6:1", 96 << 10, expect_dead=(3, 6))
    assert codes[3] == 1 and codes[6] == 1, codes
    assert [r[0] for r in res] == [0, 1, 2, 4, 5, 7] and all(r[1] == "ok" for r in res), res
    for _, _, got, st in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert st["recovered_ranks"] == 2 and st["world"] == 6
    assert dt < 170, dt


def _store_worker(rank, world_size, port, repo, q, fault):
    """Like _elastic_worker, with the rendezvous store hosted by the test process (as torchrun's
    agent hosts it), so that rank 0 may die too."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZEST_SWARM_FAULT=fault,
                      ZEST_SWARM_CTL_TIMEOUT="20", ZEST_SWARM_HB_STALE="3")
    store = dist.TCPStore("127.0.0.1", port, world_size, is_master=False)
    dist.init_process_group("gloo", store=store, rank=rank, world_size=world_size)
    from zest_amd.parallel import swarm_pull
    st = {}
    try:
        t = swarm_pull(repo, p2p=False, dht=False, stats=st, round_bytes=256 << 10)
        q.put((rank, "ok", {k: v.contiguous().view(torch.uint8).numpy().tobytes() for k, v in t.items()}, st))
    except Exception as e:
        q.put((rank, type(e).__name__, str(e), st))


def test_swarm_pull_survives_losing_the_planning_rank(hub_env):
    """Rank 0 lists the repository and makes the plan; here it dies doing so.  The others wait for
    the plan only while rank 0's heartbeat is fresh, then rebuild their groups without it, and the
    next survivor plans: ranks 1 and 2 end with every tensor."""
    import queue as _q
    world, hub = hub_env
    want = _expected(world)
    port = free_port()
    store = torch.distributed.TCPStore("127.0.0.1", port, 3, is_master=True, wait_for_workers=False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_store_worker, args=(r, 3, port, world.spec.repo_id, q, "exit:0:-1")) for r in range(3)]
    for p in procs:
        p.start()
    res = []
    for _ in range(2):
        try:
            res.append(q.get(timeout=180))
        except _q.Empty:
            break
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    del store
    res.sort(key=lambda r: r[0])
    assert procs[0].exitcode == 1
    assert [r[0] for r in res] == [1, 2] and [r[1] for r in res] == ["ok", "ok"], res
    for _, _, got, st in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert st["world"] == 2


def test_swarm_plan_term_shares_and_jobs():
    """The plan behind swarm_pull: files laid out 4 KiB aligned in one arena, byte-balanced contiguous
    term shares per rank, rounds cut by bytes with the head/tail taper, and a round item spanning two
    files turned into one fetch job per file with consecutive chunk indices."""
    import numpy as np

    from zest_amd.parallel.swarm_pull import _Plan, round_weights, split_bytes
    files = [{"path": "a.safetensors", "size": 10_000, "xet_hash": "a" * 64},
             {"path": "b.safetensors", "size": 7_000, "xet_hash": "b" * 64}]
    shapes = [[(4000, 2), (6000, 3)], [(3000, 1), (4000, 4)]]
    P = _Plan(files, shapes)
    assert P.file_off == [0, 12288] and P.arena_bytes == 12288 + 8192
    assert P.t_dst.tolist() == [0, 4000, 12288, 15288] and P.t_c0.tolist() == [0, 2, 5, 6] and P.n_chunks == 10
    assert P.region(1, 3) == (4000, 15288)
    jobs = P.jobs(1, 4, 1 << 40)
    assert jobs == [("a" * 64, 1, 2, (1 << 40) + 4000, 2), ("b" * 64, 0, 2, (1 << 40) + 12288, 5)]
    assert P.files_of(1, 3) == [0, 1]
    # shares and rounds
    ulen = np.array([100] * 40, dtype=np.int64)
    assert split_bytes(ulen, 0, 40, [1.0, 1.0]) == [(0, 20), (20, 40)]
    assert split_bytes(ulen, 5, 5, [1.0, 1.0]) == [(5, 5), (5, 5)]
    w = round_weights(10 << 30, 1 << 30)
    assert w[:2] == [0.25, 0.5] and w[-3:] == [0.5, 0.25, 0.125] and abs(sum(w) - 10) < 1.0
    assert round_weights(3 << 30, 1 << 30) == [1.0, 1.0, 1.0]
    cuts = split_bytes(ulen, 0, 40, w)
    assert cuts[0][0] == 0 and cuts[-1][1] == 40 and all(a <= b for a, b in cuts)


def test_assign_owners_follows_possession():
    """Ownership follows possession: nothing held -> the byte-balanced contiguous
    split; one rank holding everything -> it owns every term (the node's seeder); every rank holding
    everything (a shared node cache) -> balanced again; partial holdings -> holders own what they
    hold and the rest is water-filled so totals even out."""
    import numpy as np

    from zest_amd.parallel.swarm_pull import assign_owners, rank_items
    ulen = np.full(12, 100, dtype=np.int64)
    assert assign_owners(ulen, None, 3).tolist() == [0] * 4 + [1] * 4 + [2] * 4
    held = np.zeros((3, 12), dtype=bool)
    held[0] = True
    assert assign_owners(ulen, held, 3).tolist() == [0] * 12
    assert assign_owners(ulen, np.ones((3, 12), dtype=bool), 3).tolist() == [0] * 4 + [1] * 4 + [2] * 4
    held = np.zeros((3, 12), dtype=bool)
    held[2, :6] = True          # rank 2 holds the first half
    own = assign_owners(ulen, held, 3)
    assert (own[:6] == 2).all()
    # the other half goes to ranks 0 and 1 (rank 2 is already at half the model)
    assert set(own[6:].tolist()) <= {0, 1} and sorted(np.bincount(own, minlength=3).tolist()) == [3, 3, 6]
    # items: contiguous ranges, cut into rounds and at the gaps of a rank's share
    own = np.array([0, 0, 1, 1, 0, 0, 0, 1, 1, 1, 0, 0])
    assert rank_items(ulen, own, 0, [1.0]) == [(0, 2), (4, 7), (10, 12)]
    assert rank_items(ulen, own, 1, [1.0, 1.0]) == [(2, 4), (7, 8), (8, 10)]
    assert rank_items(ulen, own, 2, [1.0]) == []


def _warm_worker(rank, world_size, port, repo, q, cache_dirs):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZEST_CACHE_DIR=cache_dirs[rank])
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from zest_amd.parallel import swarm_pull
        st = {}
        try:
            t = swarm_pull(repo, p2p=False, dht=False, stats=st)
            q.put((rank, "ok", {k: v.contiguous().view(torch.uint8).numpy().tobytes() for k, v in t.items()}, st))
        except Exception as e:
            q.put((rank, type(e).__name__, str(e), st))
    finally:
        dist.destroy_process_group()


def _run_warm(world_size, repo, cache_dirs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_warm_worker, args=(r, world_size, port, repo, q, cache_dirs))
             for r in range(world_size)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_swarm_pull_warm_rank_seeds_the_node(hub_env, tmp_path):
    """BASELINE config 2 on the public path (1 seeder + N leechers): rank 0's xorb cache already
    holds the model (an earlier pull), ranks 1 and 2 start cold.  The possession have-map makes rank
    0 own every term: it reads them from its cache and the others receive everything over the
    exchange -- no rank touches the CDN, and every rank still verifies every tensor."""
    world, hub = hub_env
    want = _expected(world)
    dirs = [str(tmp_path / f"cache{r}") for r in range(3)]
    first = _run_warm(1, world.spec.repo_id, dirs[:1])          # rank 0 warms its cache from the CDN
    assert first[0][1] == "ok", first
    before = hub.counters.get("xorb_get", 0)
    res = _run_warm(3, world.spec.repo_id, dirs)
    assert [r[1] for r in res] == ["ok"] * 3, res
    total = sum(f.size for f in world.xet_files)
    for _, _, got, st in res:
        assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        assert st["possession"][0] == total and st["possession"][1:] == [0, 0]
    assert hub.counters.get("xorb_get", 0) == before, "a rank fetched from the CDN"
    r0, r1, r2 = (r[3] for r in res)
    assert r0["from_cache"] == total and r0["from_cdn"] == 0 and r0["fetched_bytes"] == total
    assert r1["fetched_bytes"] == 0 and r2["fetched_bytes"] == 0
    assert r1["received_bytes"] == total and r2["p2p_ratio"] == 1.0


def _mem_origin_worker(q, seed, compressed):
    """A one-rank swarm_pull whose CDN is an in-process memory origin (mem:// fetch_info URLs),
    served from a DevicePuller's origin layout -- the shape of bench.py's swarm row, on the CPU."""
    import tempfile

    import torch.distributed as dist

    from zest_amd import ops
    from zest_amd.engine import DevicePuller
    from zest_amd.parallel import swarm_pull
    from zest_amd.testing import FakeHub
    try:
        world = _sharded_world(seed)
        contents = world.build_on_host()
        arena = torch.zeros(world.arena_bytes + 4096, dtype=torch.uint8)[: world.arena_bytes]
        puller = DevicePuller(world, arena, 0, 1, round_bytes=1 << 20)
        puller.build_origin_host(contents)
        hub = FakeHub()
        hub.xorb_url = "mem://origin"
        hub.start()
        hub.add_world(world, exact=True, payload=False)
        T = world.terms
        ops.mem_origin_add([world.xorb_hash_hex(int(T["xorb"][t])) for t in range(len(T))],
                           [int(T["ser0"][t]) for t in range(len(T))],
                           [puller.origin.ptr + int(puller.term_origin_off[t]) for t in range(len(T))],
                           [int(T["ser_len"][t]) for t in range(len(T))])
        for k, v in hub.env(tempfile.mkdtemp()).items():
            os.environ[k] = v
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
        st = {}
        t = swarm_pull(world.spec.repo_id, p2p=False, dht=False, stats=st, reuse_pipeline=True, reuse_arena=True)
        got = {k: v.contiguous().view(torch.uint8).numpy().tobytes() for k, v in t.items()}
        base = next(iter(t.values())).untyped_storage().data_ptr()
        del t
        st2 = {}
        t2 = swarm_pull(world.spec.repo_id, p2p=False, dht=False, stats=st2, reuse_pipeline=True, reuse_arena=True)
        got2 = {k: v.contiguous().view(torch.uint8).numpy().tobytes() for k, v in t2.items()}
        st2["same_arena"] = next(iter(t2.values())).untyped_storage().data_ptr() == base
        del t2
        from zest_amd.parallel.swarm_pull import release_pipelines
        release_pipelines()
        st2["got2_equal"] = got2 == got
        q.put(("ok", got, st, st2, hub.counters.get("xorb_get", 0), hub.counters.get("cas_v1", 0)))
        dist.destroy_process_group()
        hub.stop()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((type(e).__name__, traceback.format_exc(), None, None, 0, 0))


def test_swarm_pull_from_memory_origin_and_pipeline_reuse():
    """The bench's public-path row on the CPU: fetch_info URLs mem://origin/<xorb> are served from
    registered host memory (no sockets, no xorb GETs), every tensor arrives intact, and a second pull
    with reuse_pipeline=True reuses the first one's pipelines but asks the CAS for the
    reconstructions again; with reuse_arena=True it lands in the first pull's arena."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_mem_origin_worker, args=(q, 21, False))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] == "ok", res[1]
    _, got, st, st2, xorb_gets, cas_calls = res
    want = _expected(_sharded_world(21))
    assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
    assert xorb_gets == 0  # every byte came from the memory origin
    assert st["from_cdn"] == st["total_bytes"] and not st["reused_pipeline"] and st2["reused_pipeline"]
    # reuse_arena: the second pull lands in the first one's arena, and intact
    assert not st["alloc"].get("reused") and st2["alloc"].get("reused") and st2["same_arena"] and st2["got2_equal"]
    # a reused pipeline reports this pull's bytes, not the session's running total (the second pull
    # finds the first one's runs in its xorb cache: possession makes it read them from there)
    src = ("bytes_from_cdn", "bytes_from_cache", "bytes_from_peer")
    assert sum(st2["fetch_stats"][k] for k in src) == sum(st["fetch_stats"][k] for k in src) > 0
    assert st2["from_cache"] == st2["total_bytes"] and st2["possession"] == [st2["total_bytes"]]
    n_files = st["files"]
    assert cas_calls >= 2 * n_files  # reconstructions fetched anew by the second pull


def _stuck_recovery_worker(rank, world_size, port, repo, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ZEST_SWARM_FAULT="exit:2:1",
                      ZEST_SWARM_CTL_TIMEOUT="20", ZEST_SWARM_HB_STALE="3", ZEST_SWARM_FAULT_RECOVER="hang",
                      ZEST_SWARM_RECOVER_TIMEOUT="8")
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    from zest_amd.parallel import swarm_pull
    try:
        swarm_pull(repo, p2p=False, dht=False, round_bytes=256 << 10)
        q.put((rank, "ok"))
    except Exception as e:
        q.put((rank, type(e).__name__))


def test_swarm_pull_stuck_recovery_exits_in_bounded_time(hub_env):
    """the recovery after a lost rank (RCCL abort, device synchronize, new groups) runs
    under a deadline.  Here rank 2 dies and the survivors' recovery is stubbed to hang: each exits
    with status 3 once ZEST_SWARM_RECOVER_TIMEOUT passes, instead of waiting forever."""
    import time as _t
    world, hub = hub_env
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_stuck_recovery_worker, args=(r, 3, port, world.spec.repo_id, q)) for r in range(3)]
    t0 = _t.monotonic()
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=150)
    dt = _t.monotonic() - t0
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [3, 3, 1], codes
    assert q.empty()  # nobody returned from the pull
    assert dt < 120, dt


def test_single_command_replicated_pull(hub_env, tmp_path):
    """`python -m zest_amd pull <repo> --gpus 3 --device all --save-snapshot` (here --cpu: host
    memory, gloo): one command starts 3 rank processes, every rank ends with every tensor verified,
    each prints its status line, and rank 0 writes the HF-cache snapshot once."""
    import subprocess
    import sys

    world, hub = hub_env
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "zest_amd", "pull", world.spec.repo_id, "--gpus", "3", "--device", "all", "--cpu",
           "--save-snapshot", "--no-p2p", "--no-dht", "--round-mb", "1", "--timeout", "240"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=root))
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("[rank ")]
    assert len(lines) == 3 and all("tensors" in ln and "verified" in ln for ln in lines), r.stdout
    n_t = len(_expected(world))
    assert all(f"{n_t} tensors" in ln for ln in lines), lines
    snaps = sorted((tmp_path / "hf").rglob("snapshots/*/*.safetensors"))
    assert {p.name for p in snaps} == {os.path.basename(f.path) for f in world.xet_files}
    for f in world.xet_files:
        p = next(x for x in snaps if x.name == os.path.basename(f.path))
        assert p.read_bytes() == world.file_bytes_host(f)
