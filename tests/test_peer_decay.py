"""A discovered peer that answered NOT_FOUND early (it was still pulling the same model) is tried
again once its miss window decays (ZEST_PEER_MISS_DECAY_S): the second pull of the same process
gets the bytes from it instead of the CDN.  Without the decay the peer stays skipped for the life
of the process (csrc/core/swarm.cpp miss counters never decayed)."""
from __future__ import annotations

import time

from e2e_util import free_port
from zest_amd import _core
from zest_amd.testing import FakeHub


def _files():
    import numpy as np
    rng = np.random.default_rng(5)
    return {"model.safetensors": rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()}


def test_peer_misses_decay(tmp_path, monkeypatch):
    hub = FakeHub(max_xorb_bytes=128 << 10)
    hub.start()
    try:
        repo = "org/decay"
        files = _files()
        hub.add_repo(repo, files, xet_min_size=1)
        assert len(hub.xorbs) >= 12  # enough terms for the peer to collect >= 8 misses
        for k, v in hub.env(str(tmp_path / "leech")).items():
            monkeypatch.setenv(k, v)
        # the seeder: an (initially empty) xorb cache of its own behind a BT listener
        monkeypatch.setenv("ZEST_CACHE_DIR", str(tmp_path / "seed"))
        seeder = _core.Seeder(0)
        # it is discovered through the hub's tracker for every xorb
        with hub.lock:
            for x in hub.xorbs:
                hub.tracker_peers[_core.info_hash(_core.from_xet_hex(x.hash_hex))] = {f"127.0.0.1:{seeder.port}": time.time()}
        monkeypatch.setenv("ZEST_CACHE_DIR", str(tmp_path / "leech" / "zest"))
        monkeypatch.setenv("ZEST_CACHE_WRITES", "0")        # the leecher never reads its own cache
        monkeypatch.setenv("ZEST_PEER_MISS_DECAY_S", "1")
        monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
        f = _core.HostXetFetcher(repo, p2p=True, tracker=hub.url + "/announce", dht=False, concurrency=2)
        xh = hub.xet_hash(repo, "model.safetensors")
        n = len(files["model.safetensors"])
        import numpy as np
        out = np.zeros(n, dtype=np.uint8)
        f.fetch_files([(xh, out.ctypes.data, n)])
        import json
        st = json.loads(f.stats_json())
        assert st["bytes_from_peer"] == 0 and st["bytes_from_cdn"] > 0
        assert seeder.stats()["not_found"] >= 8
        # now the seeder has every xorb
        monkeypatch.setenv("ZEST_CACHE_DIR", str(tmp_path / "seed"))
        for x in hub.xorbs:
            _core.cache_put_xorb(x.hash_hex, x.data)
        seeder.rescan()
        time.sleep(1.2)  # past the miss window
        out[:] = 0
        f.fetch_files([(xh, out.ctypes.data, n)])
        st2 = json.loads(f.stats_json())
        assert st2["bytes_from_peer"] > 0, st2
        assert out.tobytes() == files["model.safetensors"]
    finally:
        hub.stop()
