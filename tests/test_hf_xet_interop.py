"""Interop with the official Xet client: hf_xet (xet-core) downloads files from the fake CAS whose
xorbs, chunk hashes, Merkle/file hashes and LZ4/BG4 chunk payloads are produced entirely by this
framework's codec.  hf_xet verifies everything it reads, so a byte-exact download proves the
serialization and hashing are wire-compatible (the reverse direction — our reader on xorbs written
by hf_xet — is in test_xet_golden.py)."""
from __future__ import annotations

import os
import time

import numpy as np
import pytest

from zest_amd.testing import FakeHub

hf_xet = pytest.importorskip("hf_xet")


@pytest.mark.parametrize("policy", ["none", "lz4", "bg4", "auto"])
def test_hf_xet_downloads_our_xorbs(policy, tmp_path):
    rng = np.random.default_rng(5)
    w = (rng.standard_normal(700_000).astype(np.float32) * 0.02).view(np.uint32) >> 16
    files = {
        "random.bin": rng.integers(0, 256, 2_500_000, dtype=np.uint8).tobytes(),
        "periodic.bin": (bytes(range(256)) * 6000)[:1_400_000],   # dedups to a few 128 KiB chunks
        "weights.bin": w.astype(np.uint16).tobytes(),              # bf16-like: BG4 territory
    }
    hub = FakeHub(policy=policy, max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_repo("org/interop", files)
        infos = [hf_xet.PyXetDownloadInfo(str(tmp_path / n), hub.xet_hash("org/interop", n), len(d))
                 for n, d in files.items()]
        hf_xet.download_files(infos, hub.url, ("xet-" + hub.token, int(time.time()) + 3600), None, None)
        for n, d in files.items():
            assert (tmp_path / n).read_bytes() == d, n
        assert hub.counters.get("cas_v1", 0) >= len(files)
    finally:
        hub.stop()
