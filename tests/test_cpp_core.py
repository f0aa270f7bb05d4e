"""Native C++ unit tests (tests/cpp/core_tests.cpp) and host sanitizer passes.

The ASan build (python tools/build.py --asan -> build/asan/) compiles the whole host core with
-fsanitize=address,undefined and the TSan build (--tsan -> build/tsan/) with -fsanitize=thread; the
native unit tests and a real CLI pull + loopback P2P session (server threads, parallel downloader
pool, peer pool, announce thread) run under each (the reference has no sanitizers
configured and its concurrent stats/pool code has data races, items a-f)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

from e2e_util import Node, assert_snapshot, p2p_ratio, sample_files
from zest_amd.testing import FakeHub

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _build(**kw):
    from tools.build import build

    return build(**kw)


def test_native_unit_tests():
    out = _build(only="tests")["tests"]
    r = subprocess.run([str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


SAN_ENV = {
    "asan": {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1"},
    "tsan": {"TSAN_OPTIONS": "halt_on_error=1:abort_on_error=1:second_deadlock_stack=1"},
}
SAN_REPORTS = ("ERROR: AddressSanitizer", "runtime error", "WARNING: ThreadSanitizer")


@pytest.fixture(scope="module", params=["asan", "tsan"])
def san_build(request):
    if os.environ.get("ZEST_SKIP_ASAN") == "1":
        pytest.skip("ZEST_SKIP_ASAN=1")
    return request.param, _build(**{request.param: True})


def test_native_unit_tests_sanitized(san_build):
    san, b = san_build
    env = dict(os.environ, **SAN_ENV[san])
    if san == "asan":
        env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    r = subprocess.run([str(b[f"{san}_tests"])], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert not any(m in r.stderr for m in SAN_REPORTS), r.stderr[-4000:]


def test_cli_pull_and_p2p_sanitized(san_build, tmp_path):
    san, b = san_build
    zest = str(b[f"{san}_cli"])
    env_extra = SAN_ENV[san]
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        files = sample_files(seed=8)
        commit = hub.add_repo("org/san", files, xet_min_size=100_000)
        a = Node(hub, tmp_path, "a")
        r = subprocess.run([zest, "pull", "org/san", "--no-p2p"], env=dict(a.env, **env_extra), capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
        assert not any(m in r.stderr for m in SAN_REPORTS), r.stderr[-4000:]
        assert_snapshot(a, "org/san", commit, files)
        srv = subprocess.Popen([zest, "serve", "--listen-port", str(a.listen_port), "--http-port", str(a.http_port)],
                               env=dict(a.env, **env_extra), stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                               text=True)
        a.procs.append(srv)
        a.wait_healthy(30)
        b_ = Node(hub, tmp_path, "b")
        r = subprocess.run([zest, "pull", "org/san", "--peer", f"127.0.0.1:{a.listen_port}", "--no-dht"],
                           env=dict(b_.env, **env_extra), capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
        assert not any(m in r.stderr for m in SAN_REPORTS), r.stderr[-4000:]
        assert p2p_ratio(r.stdout) == 100.0
        assert_snapshot(b_, "org/san", commit, files)
        a.api("/v1/stop", "POST")
        srv.wait(timeout=30)
        out = srv.stdout.read()
        assert srv.returncode == 0 and not any(m in out for m in SAN_REPORTS), out[-4000:]
        b_.close()
        a.close()
    finally:
        hub.stop()
