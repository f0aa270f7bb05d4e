"""GPU: snapshot → HBM loading with on-device Xet verification (CDC + BLAKE3 + Merkle kernels),
compared against the host (C++) Xet implementation, which is itself pinned to hf_xet."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest
import torch

from e2e_util import free_port
from zest_amd import _core, models
from zest_amd import device as zdev
from zest_amd.synthetic import SyntheticWorld
from zest_amd.testing import FakeHub

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 63, 8191, 8192, 8193, 131072, 131073, 1 << 20, 3_000_017])
def test_xet_file_hash_device_matches_host(n):
    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, n, dtype=np.uint8)
    if n > 200_000:
        data[n // 3: n // 3 + 150_000] = 7  # long constant run: forces max-size cuts
    host = _core.xet_hex(_core.xet_file_hash(data))
    buf = torch.from_numpy(data).to("cuda:0")
    assert zdev.xet_file_hash(buf) == host


def test_pull_to_device(tmp_path, monkeypatch):
    import zest_amd

    world = SyntheticWorld(models.get("llama-tiny"), seed=11, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
        tensors = zest_amd.pull(world.spec.repo_id, device="cuda:0", p2p=False)
        host = zdev.load_snapshot(zest_amd.pull(world.spec.repo_id, p2p=False), "cpu")
        assert set(tensors) == set(host)
        for k, t in tensors.items():
            assert t.device.type == "cuda"
            assert torch.equal(t.cpu().view(torch.uint8), host[k].view(torch.uint8))
        # tamper on disk -> device verification must fail
        snap = zest_amd.pull(world.spec.repo_id, p2p=False)
        res = zest_amd.client.ZestClient().pull_detailed(world.spec.repo_id, p2p=False)
        p = os.path.join(snap, world.xet_files[0].path)
        with open(p, "r+b") as fh:
            fh.seek(100_000)
            b = fh.read(1)
            fh.seek(100_000)
            fh.write(bytes([b[0] ^ 0x80]))
        with pytest.raises(zdev.VerifyError):
            zdev.load_snapshot(snap, "cuda:0", res.xet_hashes())
    finally:
        hub.stop()


@pytest.mark.parametrize("policy", ["none", "lz4", "bg4", "auto"])
def test_direct_pull_to_device(tmp_path, monkeypatch, policy):
    """Network -> HBM with GPU decode + Merkle verify (no disk), incl. P2P from a local seeder."""
    import zest_amd
    from e2e_util import Node

    world = SyntheticWorld(models.get("llama-tiny"), seed=12, mode="bf16")
    hub = FakeHub(policy=policy, max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path / "a")).items():
            monkeypatch.setenv(k, v)
        monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
        got = zest_amd.pull(world.spec.repo_id, device="cuda:0", direct=True, p2p=False)
        host = zdev.load_snapshot(zest_amd.pull(world.spec.repo_id, p2p=False), "cpu")
        assert set(got) == set(host)
        for k, t in got.items():
            assert t.device.type == "cuda" and torch.equal(t.cpu().view(torch.uint8), host[k].view(torch.uint8))
        # P2P: node "a" (which now has the xorbs cached) seeds, a fresh node pulls to HBM from it
        seeder = Node(hub, tmp_path, "seed-a")
        seeder.env.update(hub.env(str(tmp_path / "a")))
        seeder.env["ZEST_LISTEN_PORT"] = str(seeder.listen_port)
        seeder.spawn("serve", "--listen-port", str(seeder.listen_port), "--http-port", str(seeder.http_port))
        seeder.wait_healthy()
        for k, v in hub.env(str(tmp_path / "b")).items():
            monkeypatch.setenv(k, v)
        before = hub.counters.get("xorb_get", 0)
        got2 = zest_amd.pull(world.spec.repo_id, device="cuda:0", direct=True, peers=[f"127.0.0.1:{seeder.listen_port}"],
                             dht=False)
        assert hub.counters.get("xorb_get", 0) == before
        for k, t in got2.items():
            assert torch.equal(t.cpu().view(torch.uint8), host[k].view(torch.uint8))
        seeder.close()
    finally:
        hub.stop()


@pytest.mark.parametrize("policy", ["none", "bg4"])
def test_direct_pull_repairs_corrupt_peer(tmp_path, monkeypatch, policy):
    """A corrupt seeder: the device-direct pull catches the bad bytes in the GPU Merkle check (or the
    GPU decoder), drops the quarantined peer runs and pulls the file again from the CDN; the leecher's
    xorb cache ends up holding only verified runs (a cache-only re-pull is exact)."""
    import zest_amd
    from e2e_util import Node

    world = SyntheticWorld(models.get("llama-tiny"), seed=13, mode="bf16")
    hub = FakeHub(policy=policy, max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path / "a")).items():
            monkeypatch.setenv(k, v)
        host = zdev.load_snapshot(zest_amd.pull(world.spec.repo_id, p2p=False), "cpu")
        seeder = Node(hub, tmp_path, "seed-a")
        seeder.env.update(hub.env(str(tmp_path / "a")))
        seeder.spawn("serve", "--listen-port", str(seeder.listen_port), "--http-port", str(seeder.http_port),
                     "--fault", "corrupt:1.0")
        seeder.wait_healthy()
        for k, v in hub.env(str(tmp_path / "b")).items():
            monkeypatch.setenv(k, v)
        got = zest_amd.pull(world.spec.repo_id, device="cuda:0", direct=True,
                            peers=[f"127.0.0.1:{seeder.listen_port}"], dht=False)
        for k, t in got.items():
            assert torch.equal(t.cpu().view(torch.uint8), host[k].view(torch.uint8)), k
        seeder.close()
        xorbs = tmp_path / "b" / "zest" / "xorbs"
        assert not [p for p in xorbs.rglob("*.unverified")]
        hub.fail_xorbs.update(x.hash_hex for x in hub.xorbs)  # CDN dead: only the cache can serve
        again = zest_amd.pull(world.spec.repo_id, device="cuda:0", direct=True, p2p=False)
        for k, t in again.items():
            assert torch.equal(t.cpu().view(torch.uint8), host[k].view(torch.uint8)), k
    finally:
        hub.stop()


def test_cli_bench_gpu(tmp_path):
    """`zest bench --gpu --json`: device rows in the reference bench's JSON schema."""
    import json
    import subprocess

    from e2e_util import ZEST

    env = dict(os.environ, ZEST_GPUBENCH_MIB="64")
    r = subprocess.run([str(ZEST), "bench", "--gpu", "--json"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    names = [row["name"] for row in out["results"]]
    assert names == ["blake3_64kb_gpu", "blake3_cdc_gpu", "sha1_info_hash_gpu", "cdc_gpu", "xorb_verify_gpu", "lz4_decode_gpu",
                     "lz4_decode_gpu_hostidx", "merkle_gpu", "h2d_pinned_gpu"]
    for row in out["results"]:
        assert set(row) == {"name", "runs", "median_ns", "throughput_mbps", "bytes_processed"}
        assert row["median_ns"] > 0 and row["throughput_mbps"] > 0


@pytest.mark.parametrize("worker,gpus", [("native", "1"), ("python", "1"), ("native", "0,0")])
def test_cli_pull_gpus(tmp_path, worker, gpus):
    """`zest pull <repo> --gpus N`: the CLI starts one worker per device (the native
    zest-gpu-worker, or the Python fallback) that decodes + verifies its Xet files on the GPU and
    writes them into the HF snapshot, while the CLI fetches the regular files.  `0,0` runs two
    workers on the one GPU of the test box (LPT split of the files, two status files)."""
    from e2e_util import Node, assert_snapshot, sample_files

    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        files = sample_files(seed=6)
        files["model-00002.safetensors"] = sample_files(seed=7, big=2_000_000)["model.safetensors"]
        commit = hub.add_repo("org/gpus", files, xet_min_size=100_000)
        n = Node(hub, tmp_path, "a")
        env = {"ZEST_GPU_WORKER_MODULE": "zest_amd.multigpu", "ZEST_PYTHON": sys.executable} if worker == "python" else {}
        r = n.run("pull", "org/gpus", "--gpus", gpus, "--no-p2p", timeout=300, env=env)
        n_gpus = len(gpus.split(","))
        assert f"verified on {n_gpus} GPU(s)" in r.stdout and "Done! Model available at:" in r.stdout, r.stdout + r.stderr
        if worker == "native":
            assert "[xet]" in r.stdout and "verified on the GPU" in r.stdout
        assert_snapshot(n, "org/gpus", commit, files)
        assert (n.root / "hf/hub/models--org--gpus/refs/main").read_text().strip() == commit
        # a second pull finds every Xet file verified in the cache
        r = n.run("pull", "org/gpus", "--gpus", gpus, "--no-p2p", timeout=300, env=env)
        assert r.stdout.count("(cached)") >= 2, r.stdout
        n.close()
    finally:
        hub.stop()


@pytest.mark.parametrize("staging", [64 << 10, 3 << 20])
def test_direct_pull_staging_sizes(tmp_path, monkeypatch, staging):
    """Batches are cut by a per-term byte bound; a term larger than the staging buffer grows it."""
    from zest_amd.direct import pull_to_device

    world = SyntheticWorld(models.get("llama-tiny"), seed=13, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        got = pull_to_device(world.spec.repo_id, device="cuda:0", p2p=False, staging_bytes=staging, threads=4)
        host = zdev.load_snapshot(zest_amd_pull_cpu(world.spec.repo_id), "cpu")
        assert set(got) == set(host)
        for k, t in got.items():
            assert torch.equal(t.cpu().view(torch.uint8), host[k].view(torch.uint8))
    finally:
        hub.stop()


def zest_amd_pull_cpu(repo):
    import zest_amd

    return zest_amd.pull(repo, p2p=False)


def test_pull_files_multi_file_pipeline(tmp_path, monkeypatch):
    """DeviceXetPull.pull_files: several files through one pipeline (tiny staging so batches cross
    file boundaries); a wrong expected hash is reported as a mismatch."""
    from zest_amd import _core, ops as zops

    files = {f"model-{i:05d}.safetensors": bytes(np.random.default_rng(i).integers(0, 256, 300_000 + 7919 * i,
                                                                                   dtype=np.uint8))
             for i in range(4)}
    hub = FakeHub(policy="auto", max_xorb_bytes=256 << 10)
    hub.start()
    try:
        hub.add_repo("org/multi", files, xet_min_size=1)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        commit, listing = _core.list_repo_files("org/multi", "main", "model")
        listing = sorted((f for f in listing if f["xet_hash"]), key=lambda f: f["path"])
        dp = zops.hip().DeviceXetPull("org/multi", "main", "model", False, [], None, False, [], 0, 128 << 10, 4)
        bufs = [zops.padded_empty(f["size"], "cuda:0")[:f["size"]] for f in listing]
        torch.cuda.synchronize()
        st = dp.pull_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in zip(listing, bufs)])
        assert len(st) == 4
        for f, b in zip(listing, bufs):
            assert b.cpu().numpy().tobytes() == files[f["path"]]
        wrong = listing[1]["xet_hash"][::-1]
        with pytest.raises(Exception):
            dp.pull_files([(listing[0]["xet_hash"], bufs[0].data_ptr(), listing[0]["size"]),
                           (wrong, bufs[1].data_ptr(), listing[1]["size"])])
    finally:
        hub.stop()


def test_device_pull_sibling_pipelines_and_write_behind_cache(tmp_path, monkeypatch):
    """DeviceXetPull with 3 staging slots (copy stream || kernels, event-ordered slot reuse) and a
    sibling pipeline (own streams + staging, the same Xet session / reconstructions): both pull
    byte-exact.  CDN runs reach the xorb cache through the write-behind queue (not the fetch
    threads): after flush_cache_writes() a new pipeline pulls everything from the cache with the CDN
    refusing every xorb."""
    import json as _json

    from zest_amd import _core, ops as zops

    files = {f"model-{i:05d}.safetensors": bytes(np.random.default_rng(40 + i).integers(0, 256, 250_000 + 4099 * i,
                                                                                        dtype=np.uint8))
             for i in range(4)}
    hub = FakeHub(policy="auto", max_xorb_bytes=128 << 10)
    hub.start()
    try:
        hub.add_repo("org/sib", files, xet_min_size=1)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        commit, listing = _core.list_repo_files("org/sib", "main", "model")
        listing = sorted((f for f in listing if f["xet_hash"]), key=lambda f: f["path"])
        monkeypatch.setenv("ZEST_DEVICE_TIMING", "1")
        dp = zops.hip().DeviceXetPull("org/sib", "main", "model", False, [], None, False, [], 0, 96 << 10, 4, 3)
        sib = dp.sibling(64 << 10, 2)
        bufs = [zops.padded_empty(f["size"], "cuda:0")[:f["size"]] for f in listing]
        torch.cuda.synchronize()
        dp.pull_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in zip(listing[:2], bufs[:2])])
        sib.pull_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in zip(listing[2:], bufs[2:])])
        for f, b in zip(listing, bufs):
            assert b.cpu().numpy().tobytes() == files[f["path"]]
        tl = _json.loads(dp.timeline_json())  # timed events around every batch's copy and kernels
        assert tl["batches"] >= 2 and tl["h2d_busy_ms"] > 0 and tl["kernel_busy_ms"] > 0
        assert 0 <= tl["overlap_ms"] <= min(tl["h2d_busy_ms"], tl["kernel_busy_ms"]) + 1e-3
        dp.flush_cache_writes()
        w = _json.loads(dp.cache_writer_json())
        assert w["written_bytes"] > 0 and w["dropped_bytes"] == 0
        assert len(_core.list_cached_xorbs()) == len(hub.xorbs)
        st = _json.loads(dp.stats_json())
        assert st["bytes_from_cdn"] > 0  # one session: the sibling's fetches are counted with dp's
        del sib, dp
        hub.fail_xorbs = {x.hash_hex for x in hub.xorbs}
        dp2 = zops.hip().DeviceXetPull("org/sib", "main", "model", False, [], None, False, [], 0, 96 << 10, 4)
        for b in bufs:
            b.zero_()
        dp2.pull_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in zip(listing, bufs)])
        for f, b in zip(listing, bufs):
            assert b.cpu().numpy().tobytes() == files[f["path"]]
        assert _json.loads(dp2.stats_json())["bytes_from_cdn"] == 0
    finally:
        hub.stop()


def test_dropped_cache_runs_are_refilled_and_served(tmp_path, monkeypatch):
    """a write-behind queue with no room drops runs instead of stalling the
    device pull -- they are recorded, refetched from the CDN by flush_cache_writes() (and when the
    pipeline goes), and then every xorb of the repository is served from the cache by a `zest serve`
    seeder, byte-exact."""
    import json as _json

    from zest_amd import _core, ops as zops

    files = {f"model-{i:05d}.safetensors": bytes(np.random.default_rng(70 + i).integers(0, 256, 300_000 + 5003 * i,
                                                                                        dtype=np.uint8))
             for i in range(3)}
    hub = FakeHub(policy="auto", max_xorb_bytes=128 << 10)
    hub.start()
    try:
        hub.add_repo("org/refill", files, xet_min_size=1)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        monkeypatch.setenv("ZEST_CACHE_WRITE_QUEUE_BYTES", "1")  # every run overflows the queue
        commit, listing = _core.list_repo_files("org/refill", "main", "model")
        listing = sorted((f for f in listing if f["xet_hash"]), key=lambda f: f["path"])
        dp = zops.hip().DeviceXetPull("org/refill", "main", "model", False, [], None, False, [], 0, 1 << 20, 4)
        bufs = [zops.padded_empty(f["size"], "cuda:0")[:f["size"]] for f in listing]
        torch.cuda.synchronize()
        dp.pull_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in zip(listing, bufs)])
        for f, b in zip(listing, bufs):
            assert b.cpu().numpy().tobytes() == files[f["path"]]
        w = _json.loads(dp.cache_writer_json())
        assert w["dropped_bytes"] > 0 and w["deferred_runs"] >= len(hub.xorbs), w  # (a xorb per term)
        dp.flush_cache_writes()  # the dropped runs are fetched again and cached
        assert _json.loads(dp.cache_writer_json())["deferred_runs"] == 0
        assert len(_core.list_cached_xorbs()) == len(hub.xorbs)
        seeder = _core.Seeder(0)
        try:
            for x in hub.xorbs:
                data, off, _ = _core.peer_fetch(f"127.0.0.1:{seeder.port}", _core.from_xet_hex(x.hash_hex), 0, 0)
                # a cached run is the chunk span the pull's terms needed (a CDN range, not always the
                # whole xorb): its bytes are the xorb's serialized chunks from chunk `off` on
                b0 = x.boundaries[off - 1] if off else 0
                assert data and data == x.data[b0:b0 + len(data)], x.hash_hex
        finally:
            seeder.stop()
    finally:
        hub.stop()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_device_pull_on_second_gpu_from_another_thread(tmp_path, monkeypatch):
    """HIP's current device is per thread.  A pipeline built for the last GPU and called
    from a thread whose current device is 0 still allocates and runs on its own GPU."""
    import threading

    from zest_amd import _core, ops as zops

    data = bytes(np.random.default_rng(9).integers(0, 256, 400_000, dtype=np.uint8))
    hub = FakeHub(policy="auto", max_xorb_bytes=128 << 10)
    hub.start()
    try:
        hub.add_repo("org/dev1", {"m.safetensors": data}, xet_min_size=1)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        last = torch.cuda.device_count() - 1
        _, listing = _core.list_repo_files("org/dev1", "main", "model")
        f = [x for x in listing if x["xet_hash"]][0]
        dp = zops.hip().DeviceXetPull("org/dev1", "main", "model", False, [], None, False, [], last, 96 << 10, 4)
        buf = zops.padded_empty(f["size"], f"cuda:{last}")[:f["size"]]
        torch.cuda.synchronize(last)
        err = []

        def run():
            torch.cuda.set_device(0)
            try:
                dp.pull_files([(f["xet_hash"], buf.data_ptr(), f["size"])])
            except Exception as e:  # noqa: BLE001
                err.append(e)
        t = threading.Thread(target=run)
        t.start()
        t.join()
        assert not err, err
        assert buf.cpu().numpy().tobytes() == data
    finally:
        hub.stop()


def _swarm_pull_gpu_worker(rank, world_size, port, repo, backend, q, exchange="auto", fault="", round_bytes=None,
                           swarm_fault=""):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fault:
        os.environ["ZEST_VMM_FAULT"] = fault
    if swarm_fault:
        os.environ.update(ZEST_SWARM_FAULT=swarm_fault, ZEST_SWARM_CTL_TIMEOUT="20", ZEST_SWARM_HB_STALE="3")
    torch.cuda.set_device(0)
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world_size, **kw)
    try:
        from zest_amd.parallel import swarm_pull
        st = {}
        t = swarm_pull(repo, device="cuda:0", p2p=False, dht=False, stats=st, exchange=exchange,
                       round_bytes=round_bytes)
        assert all(v.device.type == "cuda" for v in t.values())
        q.put((rank, {k: v.contiguous().view(torch.uint8).cpu().numpy().tobytes() for k, v in t.items()}, st))
    except Exception as e:
        q.put((rank, f"{type(e).__name__}: {e}", {}))
    finally:
        if not swarm_fault:  # (the default group still counts a dead rank)
            dist.destroy_process_group()


def _swarm_repeat_worker(rank, world_size, port, repo, q):
    """Three peer-mapped (xgmi) pulls in one process: every pull gets a fresh, ordinary arena that is
    freed once its tensors are dropped; the exchange windows are mapped once (first pull) and reused;
    device memory comes back to where it was after the first pull, and a pull made while the
    previous pull's tensors are still held costs exactly one more arena."""
    import gc
    import time as _t

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from zest_amd.parallel import swarm_pull

        def pull():
            st = {}
            t = swarm_pull(repo, device="cuda:0", p2p=False, dht=False, stats=st, exchange="xgmi",
                           round_bytes=64 << 20)
            return t, st

        def host(t):
            return {k: v.contiguous().view(torch.uint8).cpu().numpy().tobytes() for k, v in t.items()}

        def free():  # device-wide free bytes once every rank is here and frees have settled
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            dist.barrier()
            last = torch.cuda.mem_get_info()[0]
            for _ in range(40):
                _t.sleep(0.05)
                f = torch.cuda.mem_get_info()[0]
                if f == last:
                    break
                last = f
            dist.barrier()
            return last
        t1, st1 = pull()
        got1 = host(t1)
        del t1
        f1 = free()
        t2, st2 = pull()
        got2 = host(t2)
        f2 = free()  # t2 held
        t3, st3 = pull()
        torch.cuda.synchronize()
        kept2 = host(t2)
        got3 = host(t3)
        f3 = free()  # t2 and t3 held
        del t2, t3
        f4 = free()
        t4, _ = pull()
        del t4
        f5 = free()  # a fourth pull, dropped: nothing accumulates pull after pull
        arena = st1["total_bytes"]
        q.put((rank, got1, [st1.get("phases", {}).get("windows_s"), st2.get("phases", {}).get("windows_s")],
               got2 == got1, kept2 == got1, got3 == got1, (f1, f2, f3, f4, f5, arena),
               [st1["exchange"], st2["exchange"], st3["exchange"]]))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc(), None, None, None, None, None, None))
    finally:
        dist.destroy_process_group()


def test_swarm_pull_arenas_are_freed_and_windows_mapped_once(tmp_path, monkeypatch):
    import dataclasses

    import torch.multiprocessing as mp

    # a ~0.5 GB model: a per-pull leak of the size of an arena (what released peer-mapped VMM arenas
    # did, profiles/r6/vmm_release_r6h_r6i/) stands out from allocator noise
    spec = dataclasses.replace(models.get("gpt2"), max_shard_bytes=200_000_000)
    world = SyntheticWorld(spec, seed=23, mode="random")
    hub = FakeHub(policy="none", max_xorb_bytes=32 << 20)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=_swarm_repeat_worker, args=(r, 2, port, world.spec.repo_id, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = [q.get(timeout=240) for _ in procs]
        for p in procs:
            p.join(timeout=60)
        for rank, got1, win_s, same2, kept2, same3, mem, modes in res:
            assert isinstance(got1, dict), got1
            assert same2 and kept2 and same3
            assert modes == ["xgmi"] * 3, modes
            f1, f2, f3, f4, f5, arena = mem
            slack = 256 << 20  # allocator granularity, tables, staging of the two ranks' pipelines
            # two ranks share the GPU: "one arena" per pull is two arenas of the device
            assert f1 - f2 <= 2 * arena + slack, mem                  # one live pull: its arenas only
            assert f2 - f3 <= 2 * arena + slack, mem                  # held tensors: one more arena each
            assert f4 >= f1 - slack and f5 >= f1 - slack, mem         # dropped: memory comes back
    finally:
        hub.stop()


@pytest.mark.parametrize("world_size,backend,exchange,fault", [
    (1, "nccl", "auto", ""), (2, "gloo", "auto", ""), (2, "gloo", "xgmi", ""), (2, "gloo", "ipc", ""),
    (2, "gloo", "allgather", ""), (2, "gloo", "auto", "import"), (2, "gloo", "auto", "sentinel"),
    (2, "gloo", "xgmi", "gather")])
def test_swarm_pull_device_direct(tmp_path, monkeypatch, world_size, backend, exchange, fault):
    """Term-sharded swarm pull into HBM: each rank fetches its term ranges device-direct (GPU decode
    + chunk hashes into the arena), the rounds are replicated to the other ranks (here: ranks sharing
    the one GPU over gloo, arenas peer-mapped through HIP VMM for ipc / xgmi) and every chunk is
    re-hashed on the receiver; Merkle file hashes on every rank.  Faults (ZEST_VMM_FAULT): a refused
    import or sentinel falls back to an RCCL exchange; a corrupting gather fails the file hashes and
    the repair pass refetches + re-sends them over a broadcast."""
    import dataclasses
    import json
    import struct

    import torch.multiprocessing as mp

    spec = dataclasses.replace(models.get("llama-tiny"), max_shard_bytes=700_000)
    world = SyntheticWorld(spec, seed=22, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=256 << 10)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
        want = {}
        for f in world.xet_files:
            data = world.file_bytes_host(f)
            (hlen,) = struct.unpack("<Q", data[:8])
            for name, ent in json.loads(data[8:8 + hlen]).items():
                if name != "__metadata__":
                    a, b = ent["data_offsets"]
                    want[name] = data[8 + hlen + a:8 + hlen + b]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=_swarm_pull_gpu_worker,
                             args=(r, world_size, port, world.spec.repo_id, backend, q, exchange, fault, 512 << 10))
                 for r in range(world_size)]
        for p in procs:
            p.start()
        res = [q.get(timeout=180) for _ in procs]
        for p in procs:
            p.join(timeout=60)
        for rank, got, st in res:
            assert isinstance(got, dict), got
            assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
        total = sum(f.size for f in world.xet_files)
        assert sum(r[2]["fetched_bytes"] for r in res) == total
        modes = {r[2]["exchange"] for r in res}
        assert len(modes) == 1, modes
        mode = modes.pop()
        if world_size == 1:
            assert mode == "none"
        elif fault in ("import", "sentinel"):
            assert mode in ("bcast", "allgather") and not any(r[2]["peer_mapped"] for r in res), res
        elif exchange != "auto":
            assert mode == exchange
        if fault == "gather":  # the corrupted receive failed the file hashes: repaired over a broadcast
            assert all(r[2]["repaired_files"] >= 1 and r[2]["repair_exchange"] == "bcast" for r in res), \
                [r[2] for r in res]
        else:
            assert all(r[2]["repaired_files"] == 0 for r in res)
        print(f"[swarm_pull {world_size}x{backend} {exchange}{'/' + fault if fault else ''}] mode {mode} "
              f"autotune {res[0][2]['exchange_autotune_s']} phases {res[0][2]['phases']}")
    finally:
        hub.stop()


@pytest.mark.parametrize("world_size", [1, 2])
def test_swarm_pull_hash_table_ordered_before_ingest(tmp_path, monkeypatch, world_size):
    """Round 5's 2.4-3.4 s stall: the hash table was zero-filled on torch's
    current stream while the native pipeline's ingest kernels -- on a stream of their own --
    already wrote chunk hashes into it; when the zero-fill ran late it wiped them, the Merkle check
    failed and the pull paid a CDN repair.  Here the current stream is held busy (~0.25 s) before the
    zero-fill: the pull must still verify on its first check (no repair)."""
    import dataclasses
    import json
    import struct

    import torch.multiprocessing as mp

    spec = dataclasses.replace(models.get("llama-tiny"), max_shard_bytes=700_000)
    world = SyntheticWorld(spec, seed=29, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=256 << 10)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
        monkeypatch.setenv("ZEST_SWARM_FAULT_SLOWZERO", "500000000")
        want = {}
        for f in world.xet_files:
            data = world.file_bytes_host(f)
            (hlen,) = struct.unpack("<Q", data[:8])
            for name, ent in json.loads(data[8:8 + hlen]).items():
                if name != "__metadata__":
                    a, b = ent["data_offsets"]
                    want[name] = data[8 + hlen + a:8 + hlen + b]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        backend = "nccl" if world_size == 1 else "gloo"
        procs = [ctx.Process(target=_swarm_pull_gpu_worker,
                             args=(r, world_size, port, world.spec.repo_id, backend, q, "auto", "", 512 << 10))
                 for r in range(world_size)]
        for p in procs:
            p.start()
        res = [q.get(timeout=180) for _ in procs]
        for p in procs:
            p.join(timeout=60)
        for rank, got, st in res:
            assert isinstance(got, dict), got
            assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
            assert st["first_verify_bad_files"] == 0 and st["repaired_files"] == 0, st
    finally:
        hub.stop()


def test_swarm_pull_device_survives_a_lost_rank(tmp_path, monkeypatch):
    """SURVEY §5.3 on the GPU: 3 ranks share the device (gloo control, peer-mapped arenas, autotuned
    exchange); rank 2 exits at its second round.  Ranks 0 and 1 detect it through the control group
    and the store heartbeats, rebuild their groups in-process, re-shard rank 2's ranges (re-sent by a
    holder or refetched) and end with every tensor verified in HBM."""
    import dataclasses
    import json
    import queue as _q
    import struct

    import torch.multiprocessing as mp

    spec = dataclasses.replace(models.get("llama-tiny"), max_shard_bytes=700_000)
    world = SyntheticWorld(spec, seed=23, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=256 << 10)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
        want = {}
        for f in world.xet_files:
            data = world.file_bytes_host(f)
            (hlen,) = struct.unpack("<Q", data[:8])
            for name, ent in json.loads(data[8:8 + hlen]).items():
                if name != "__metadata__":
                    a, b = ent["data_offsets"]
                    want[name] = data[8 + hlen + a:8 + hlen + b]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=_swarm_pull_gpu_worker,
                             args=(r, 3, port, world.spec.repo_id, "gloo", q, "auto", "", 256 << 10, "exit:2:1"))
                 for r in range(3)]
        for p in procs:
            p.start()
        res = []
        for _ in range(2):
            try:
                res.append(q.get(timeout=150))
            except _q.Empty:
                break
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        res.sort(key=lambda r: r[0])
        assert procs[2].exitcode == 1
        assert [r[0] for r in res] == [0, 1], res
        for rank, got, st in res:
            assert isinstance(got, dict), got
            assert got.keys() == want.keys() and all(got[k] == want[k] for k in want)
            assert st["recovered_ranks"] == 1 and st["world"] == 2, st
        print(f"[swarm_pull lost rank] exchange {res[0][2]['exchange']} phases {res[0][2]['phases']}")
    finally:
        hub.stop()


def _swarm_load_gpu_worker(rank, world_size, port, snap, hashes, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from zest_amd.parallel import swarm_load
        t = swarm_load(snap, device="cuda:0", xet_hashes=hashes, verify_all=True)
        assert all(v.device.type == "cuda" for v in t.values())
        q.put((rank, {k: v.contiguous().view(torch.uint8).cpu().numpy().tobytes() for k, v in t.items()}))
    except Exception as e:  # noqa: BLE001 - reported to the test
        q.put((rank, type(e).__name__))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_swarm_load_device(tmp_path, monkeypatch, corrupt):
    """swarm_load of a pulled snapshot into HBM by 2 ranks sharing the GPU (gloo): each file is read
    and GPU-verified by its owner, broadcast in rounds, re-verified by the receiver; a file failing
    its owner's hash check makes both ranks raise instead of hanging in a broadcast."""
    import dataclasses

    import torch.multiprocessing as mp
    import zest_amd
    import zest_amd.client  # noqa: F401  (submodule used below)

    spec = dataclasses.replace(models.get("llama-tiny"), max_shard_bytes=700_000)
    world = SyntheticWorld(spec, seed=23, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=256 << 10)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
        res = zest_amd.client.ZestClient().pull_detailed(world.spec.repo_id, p2p=False)
        hashes = res.xet_hashes()
        assert len(hashes) >= 3
        if corrupt:
            hashes[sorted(hashes)[-1]] = "0" * 64
        want = zdev.load_snapshot(res.snapshot_dir, "cpu")
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=_swarm_load_gpu_worker, args=(r, 2, port, res.snapshot_dir, hashes, q))
                 for r in range(2)]
        for p in procs:
            p.start()
        got = dict(q.get(timeout=180) for _ in procs)
        for p in procs:
            p.join(timeout=60)
        if corrupt:
            assert got == {0: "VerifyError", 1: "VerifyError"}
            return
        for r in range(2):
            assert isinstance(got[r], dict), got[r]
            assert got[r].keys() == want.keys()
            assert all(got[r][k] == want[k].contiguous().view(torch.uint8).numpy().tobytes() for k in want)
    finally:
        hub.stop()


@pytest.mark.parametrize("n", [1, (1 << 20) - 3, 5 * (1 << 20) + 12345])
def test_write_device_file_pipelined(tmp_path, n):
    """zest pull --gpus N snapshot writer: chunked D2H into pinned slots overlapped with pwrite."""
    from zest_amd.multigpu import write_device_file

    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    buf = torch.from_numpy(data).to("cuda:0")
    p = tmp_path / "f.bin"
    write_device_file(buf, str(p), chunk=1 << 20, slots=2)
    assert p.read_bytes() == data.tobytes()
