"""Tracing (Chrome trace JSON from C++ and Python spans) and utility helpers."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from e2e_util import Node, sample_files
from zest_amd.testing import FakeHub
from zest_amd.utils import FaultSpec, human_bytes, human_rate


def test_fault_spec():
    f = FaultSpec.parse("drop:0.25,corrupt:1,delay:5")
    assert (f.drop, f.corrupt, f.delay_ms) == (0.25, 1.0, 5)
    assert FaultSpec.parse("").drop == 0
    assert f.maybe_corrupt(b"abcd") != b"abcd"
    with pytest.raises(ValueError):
        FaultSpec.parse("explode:1")


def test_fmt():
    assert human_bytes(141_107_498_032) == "141.1 GB"
    assert human_rate(2e9, 2.0) == "1.0 GB/s"
    assert human_bytes(12) == "12 B"


def test_python_spans_to_chrome_trace(tmp_path):
    out = tmp_path / "t.json"
    code = f"""
import sys; sys.path.insert(0, {str(tmp_path.parent.parent)!r})
from zest_amd import _core
_core.trace.set_output({str(out)!r})
from zest_amd.utils import Span
with Span("test", "outer", n=3):
    with Span("test", "inner"):
        pass
_core.trace.counter("bytes", 42.0)
_core.trace.flush()
"""
    import os
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       cwd=str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    assert r.returncode == 0, r.stderr
    ev = json.loads(out.read_text())["traceEvents"]
    names = {e["name"] for e in ev}
    assert {"outer", "inner", "bytes"} <= names
    outer = next(e for e in ev if e["name"] == "outer")
    assert outer["ph"] == "X" and outer["args"] == {"n": 3}


def test_cli_pull_trace_file(tmp_path):
    hub = FakeHub(max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_repo("org/t", sample_files(seed=9), xet_min_size=100_000)
        n = Node(hub, tmp_path, "a")
        trace = tmp_path / "pull.json"
        n.run("pull", "org/t", "--no-p2p", env={"ZEST_TRACE": str(trace)})
        ev = json.loads(trace.read_text())["traceEvents"]
        assert any(e["cat"] == "cdn" and e["ph"] == "X" for e in ev)
        r = n.run("pull", "org/t", "--no-p2p", env={"ZEST_TRACE": "1"})
        assert "(cached)" in r.stdout
        n.close()
    finally:
        hub.stop()


def test_roctx_ranges_optional():
    """ZEST_ROCTX=1 turns spans into roctx ranges (dlopen'ed ROCm library); push/pop must balance
    and never fail, with or without the library."""
    import subprocess
    import sys
    code = ("from zest_amd import _core\n"
            "from zest_amd.utils.trace import Span\n"
            "on = _core.trace.roctx_enabled()\n"
            "with Span('engine', 'round 0'):\n"
            "    with Span('engine', 'inner'): pass\n"
            "print('roctx', on)\n")
    for val, want in (("1", None), ("0", "False")):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, ZEST_ROCTX=val))
        assert r.returncode == 0, r.stderr
        if want:
            assert r.stdout.strip() == f"roctx {want}"


def test_trace_path_pid_substitution(tmp_path):
    """ZEST_TRACE=...%p...: each process writes its own trace (a swarm's ranks and their seeder)."""
    code = """
from zest_amd.utils import Span
with Span("test", "one"):
    pass
"""
    env = dict(os.environ, ZEST_TRACE=str(tmp_path / "t.%p.json"))
    root = str(__import__("pathlib").Path(__file__).resolve().parents[1])
    pids = []
    for _ in range(2):
        p = subprocess.Popen([sys.executable, "-c", code], env=env, cwd=root)
        assert p.wait() == 0
        pids.append(p.pid)
    for pid in pids:
        ev = json.loads((tmp_path / f"t.{pid}.json").read_text())["traceEvents"]
        assert any(e.get("name") == "one" for e in ev)
