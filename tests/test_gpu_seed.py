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
