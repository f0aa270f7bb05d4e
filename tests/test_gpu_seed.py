"""GPU: seed mode from HBM — xorbs packed into device memory by the GPU pack kernel and served over
BEP XET by the native HbmSeeder; a `zest pull` leecher gets 100 % of the bytes from it."""
from __future__ import annotations

import pytest
import torch

from e2e_util import Node, assert_snapshot, p2p_ratio
from zest_amd import _core, models, ops
from zest_amd.seed import HbmSeedServer, HbmXorbArena
from zest_amd.synthetic import SyntheticWorld
from zest_amd.testing import FakeHub

pytestmark = pytest.mark.gpu


def test_pull_from_hbm_seeder(tmp_path):
    spec = models.get("llama-tiny")
    host_world = SyntheticWorld(spec, seed=21, max_xorb_bytes=1 << 20)
    dev_world = SyntheticWorld(spec, seed=21, max_xorb_bytes=1 << 20)
    dev = torch.device("cuda:0")
    content = ops.padded_empty(dev_world.arena_bytes, dev)
    dev_world.generate_on_device(content)
    dev_world.build_on_device(content)
    arena = HbmXorbArena(dev_world, content)
    srv = HbmSeedServer(arena)
    hub = FakeHub()
    hub.start()
    try:
        commit = hub.add_world(host_world, exact=True)
        assert sorted(arena.xorb_hex) == sorted(x.hash_hex for x in hub.xorbs)
        # direct fetch: a middle chunk run of the first xorb
        conn = _core.PeerConnection(f"127.0.0.1:{srv.port}", arena.xorb_hashes[0])
        data, off = conn.fetch(arena.xorb_hashes[0], 1, 3)
        assert off == 1 and len(_core.index_chunks(data)) == 2
        node = Node(hub, tmp_path, "leecher")
        try:
            out = node.run("pull", spec.repo_id, "--peer", f"127.0.0.1:{srv.port}", "--no-dht").stdout
            assert p2p_ratio(out) == 100.0
            assert hub.counters.get("xorb_get", 0) == 0
            files = {f.path: host_world.file_bytes_host(f) for f in host_world.files}
            assert_snapshot(node, spec.repo_id, commit, files)
        finally:
            node.close()
        st = srv.stats()
        assert st["chunk_units"] >= dev_world.n_chunks and st["not_found"] == 0
    finally:
        srv.stop()
        hub.stop()


def test_warm_seeding_from_disk_cache(tmp_path, monkeypatch):
    """`python -m zest_amd.seed`: the disk xorb cache (full and partial runs) is uploaded to HBM and
    served from there; a leecher gets everything from the GPU seeder."""
    from e2e_util import sample_files
    from zest_amd.seed import HbmCacheArena, HbmCacheSeedServer

    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        files = sample_files(seed=4)
        commit = hub.add_repo("org/warm", files, xet_min_size=100_000)
        a = Node(hub, tmp_path, "a")
        a.run("pull", "org/warm", "--no-p2p")
        for k, v in a.env.items():
            if k.startswith(("ZEST_", "HF_", "HOME")):
                monkeypatch.setenv(k, v)
        arena = HbmCacheArena("cuda:0")
        assert arena.runs and arena.used > 0
        srv = HbmCacheSeedServer(arena)
        try:
            b = Node(hub, tmp_path, "b")
            before = hub.counters.get("xorb_get", 0)
            out = b.run("pull", "org/warm", "--peer", f"127.0.0.1:{srv.port}", "--no-dht").stdout
            assert p2p_ratio(out) == 100.0 and hub.counters.get("xorb_get", 0) == before
            assert_snapshot(b, "org/warm", commit, files)
            assert srv.stats()["chunks_served"] > 0
            b.close()
        finally:
            srv.stop()
        a.close()
    finally:
        hub.stop()
