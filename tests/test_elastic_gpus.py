"""Elastic `zest pull --gpus N`: an attempt that loses a worker is retried on one GPU
fewer, and after the last GPU attempt the host pipeline finishes the pull.  The GPU workers are
replaced by tests/elastic_stub_worker.py (ZEST_GPU_WORKER_MODULE) so this runs on CPU; the real
(native) worker is covered by tests/test_gpu_device.py::test_cli_pull_gpus."""
from __future__ import annotations

import sys

from e2e_util import Node, ZEST, assert_snapshot, sample_files
from zest_amd.testing import FakeHub


def _env(tmp_path, mode):
    return {"ZEST_GPU_WORKER_MODULE": "tests.elastic_stub_worker", "ZEST_PYTHON": sys.executable,
            "ZEST_STUB_MODE": mode, "ZEST_STUB_LOG": str(tmp_path / "attempts.log"), "TMPDIR": str(tmp_path)}


def test_gpu_pull_retries_on_fewer_gpus(tmp_path):
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_repo("org/elastic", sample_files(seed=5), xet_min_size=100_000)
        n = Node(hub, tmp_path, "a")
        r = n.run("pull", "org/elastic", "--gpus", "3", env=_env(tmp_path, "lose-last"), timeout=300)
        attempts = (tmp_path / "attempts.log").read_text().split()
        assert attempts == ["3@0,1,2", "2@0,1", "1@0"], attempts
        # one worker per device, each pinned to its own device
        vis = (tmp_path / "attempts.log.vis").read_text().split()
        assert sorted(vis) == ["0", "0", "0", "1", "1", "2"], vis
        assert "retrying on 2 GPU(s)" in r.stderr and "retrying on 1 GPU(s)" in r.stderr
        assert "finishing the pull on the host" not in r.stderr
    finally:
        hub.stop()


def test_gpu_pull_falls_back_to_host(tmp_path):
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        files = sample_files(seed=5)
        commit = hub.add_repo("org/elastic", files, xet_min_size=100_000)
        n = Node(hub, tmp_path, "a")
        r = n.run("pull", "org/elastic", "--gpus", "2", "--no-p2p", env=_env(tmp_path, "always-crash"), timeout=300)
        assert (tmp_path / "attempts.log").read_text().split() == ["2@0,1", "1@0"]
        assert "finishing the pull on the host" in r.stderr
        assert_snapshot(n, "org/elastic", commit, files)
        # host fallback can be disabled
        r = n.run("pull", "org/elastic", "--gpus", "1", env=dict(_env(tmp_path, "always-crash"),
                                                                 ZEST_GPU_HOST_FALLBACK="0"), check=False)
        assert r.returncode != 0 and "finishing the pull on the host" not in r.stderr
    finally:
        hub.stop()


def test_gpu_pull_device_list_and_env_default(tmp_path):
    """`--gpus 4,6,7` pins the workers to those devices (HIP_VISIBLE_DEVICES), retries drop the
    last listed device; ZEST_GPUS supplies --gpus when the flag is absent."""
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    try:
        hub.add_repo("org/elastic", sample_files(seed=5), xet_min_size=100_000)
        n = Node(hub, tmp_path, "a")
        n.run("pull", "org/elastic", "--gpus", "4,6,7", env=_env(tmp_path, "lose-last"), timeout=300)
        log = tmp_path / "attempts.log"
        assert log.read_text().split() == ["3@4,6,7", "2@4,6", "1@4"]
        log.unlink()
        n.run("pull", "org/elastic", env=dict(_env(tmp_path, "lose-last"), ZEST_GPUS="2"), timeout=300)
        assert log.read_text().split() == ["2@0,1", "1@0"]
        log.unlink()
        n.run("pull", "org/elastic", "--gpus", "5,", env=_env(tmp_path, "lose-last"), timeout=300)
        assert log.read_text().split() == ["1@5"]  # a one-device list
    finally:
        hub.stop()
