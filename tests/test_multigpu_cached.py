"""`zest pull --gpus N` workers skip a snapshot file only when it is verified (marker or re-hash),
like the host pull (csrc/core/pull.cpp); a same-size corrupt file is pulled again."""
from __future__ import annotations

import os

from zest_amd import _core
from zest_amd.multigpu import cached_file_ok


def test_cached_file_needs_verification(tmp_path, monkeypatch):
    monkeypatch.setenv("ZEST_CACHE_DIR", str(tmp_path / "zest"))
    monkeypatch.setenv("HF_HOME", str(tmp_path / "hf"))
    data = os.urandom(300_000)
    good = tmp_path / "good.bin"
    good.write_bytes(data)
    xh = _core.xet_hash_of_file(str(good))
    f = {"path": "model.safetensors", "size": len(data), "xet_hash": xh}
    dst = tmp_path / "snap" / "model.safetensors"
    dst.parent.mkdir()
    assert not cached_file_ok("org/m", "c0ffee", f, str(dst))  # missing
    # same size, one byte flipped: not cached, and no marker gets written for it
    bad = bytearray(data)
    bad[len(bad) // 2] ^= 1
    dst.write_bytes(bytes(bad))
    assert not cached_file_ok("org/m", "c0ffee", f, str(dst))
    assert not _core.check_verified_marker("org/m", "c0ffee", f["path"], xh, str(dst))
    # the right bytes without a marker: re-hashed, accepted, marker written
    dst.write_bytes(data)
    assert cached_file_ok("org/m", "c0ffee", f, str(dst))
    assert _core.check_verified_marker("org/m", "c0ffee", f["path"], xh, str(dst))
    # a rewrite (new mtime) invalidates the marker until re-hashed
    bad_st = os.stat(dst)
    dst.write_bytes(bytes(bad))
    os.utime(dst, ns=(bad_st.st_atime_ns, bad_st.st_mtime_ns + 1_000_000))
    assert not _core.check_verified_marker("org/m", "c0ffee", f["path"], xh, str(dst))
    assert not cached_file_ok("org/m", "c0ffee", f, str(dst))
