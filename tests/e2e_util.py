"""Helpers for end-to-end tests: the `zest` binary, free ports, per-node cache roots."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import time
import urllib.request
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
ZEST = str(REPO / "zest_amd" / "_bin" / "zest")


def free_port(kind: int = socket.SOCK_STREAM) -> int:
    with socket.socket(socket.AF_INET, kind) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def sample_files(seed: int = 0, big: int = 3_000_000) -> dict[str, bytes]:
    """A small repo: a JSON config, an incompressible weights file, a compressible one in a subdir."""
    rng = np.random.default_rng(seed)
    return {
        "config.json": b'{"model_type": "llama", "hidden_size": 64}',
        "model.safetensors": rng.integers(0, 256, big, dtype=np.uint8).tobytes(),
        "sub/extra.bin": rng.integers(0, 4, 500_000, dtype=np.uint8).tobytes(),
    }


class Node:
    """One simulated machine: its own HF cache, zest cache and ports."""

    def __init__(self, hub, root: Path, name: str):
        self.root = Path(root) / name
        self.root.mkdir(parents=True, exist_ok=True)
        self.hub = hub
        self.listen_port = free_port()
        self.http_port = free_port()
        self.dht_port = free_port(socket.SOCK_DGRAM)
        self.env = dict(os.environ)
        self.env.update(hub.env(str(self.root)))
        self.env.update({"ZEST_LISTEN_PORT": str(self.listen_port), "ZEST_HTTP_PORT": str(self.http_port),
                         "ZEST_DHT_PORT": str(self.dht_port), "ZEST_CONNECT_TIMEOUT_MS": "2000"})
        self.procs: list[subprocess.Popen] = []

    def run(self, *args: str, timeout: float = 120, check: bool = True, env: dict | None = None):
        e = dict(self.env, **(env or {}))
        r = subprocess.run([ZEST, *args], env=e, capture_output=True, text=True, timeout=timeout)
        if check and r.returncode != 0:
            raise AssertionError(f"zest {' '.join(args)} failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
        return r

    def spawn(self, *args: str, env: dict | None = None) -> subprocess.Popen:
        e = dict(self.env, **(env or {}))
        p = subprocess.Popen([ZEST, *args], env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        self.procs.append(p)
        return p

    def snapshot(self, repo_id: str, commit: str) -> Path:
        return self.root / "hf" / "hub" / ("models--" + repo_id.replace("/", "--")) / "snapshots" / commit

    def xorb_files(self) -> list[Path]:
        d = self.root / "zest" / "xorbs"
        return sorted(p for p in d.rglob("*") if p.is_file()) if d.exists() else []

    def api(self, path: str, method: str = "GET", body: dict | None = None, timeout: float = 5):
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(f"http://127.0.0.1:{self.http_port}{path}", data=data, method=method)
        try:
            with urllib.request.urlopen(req, timeout=timeout) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, e.read()

    def wait_healthy(self, timeout: float = 10) -> None:
        t0 = time.time()
        while time.time() - t0 < timeout:
            try:
                if self.api("/v1/health", timeout=1)[0] == 200:
                    return
            except OSError:
                pass
            time.sleep(0.05)
        raise TimeoutError("zest server did not come up")

    def wait_port(self, port: int, timeout: float = 10) -> None:
        t0 = time.time()
        while time.time() - t0 < timeout:
            with socket.socket() as s:
                if s.connect_ex(("127.0.0.1", port)) == 0:
                    return
            time.sleep(0.05)
        raise TimeoutError(f"port {port} not listening")

    def close(self) -> None:
        for p in self.procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            if p.stdout:
                p.stdout.close()


def assert_snapshot(node: Node, repo_id: str, commit: str, files: dict[str, bytes]) -> None:
    snap = node.snapshot(repo_id, commit)
    for path, data in files.items():
        got = (snap / path).read_bytes()
        assert got == data, f"{path}: content mismatch ({len(got)} vs {len(data)} bytes)"
    assert not list(snap.rglob("*.incomplete")), "leftover .incomplete files"


def p2p_ratio(stdout: str) -> float:
    for line in stdout.splitlines():
        if line.strip().startswith("P2P ratio:"):
            return float(line.split(":")[1].strip().rstrip("%"))
    raise AssertionError("no P2P ratio line:\n" + stdout)
