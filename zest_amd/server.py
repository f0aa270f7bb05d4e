"""Lifecycle of the background `zest serve` process (BT seeder + REST API on 127.0.0.1).

Reference: python/zest/server.py:1-95 — health check on /v1/health, spawn `zest serve --http-port`,
poll every 0.2 s for up to 5 s, stop via POST /v1/stop, binary lookup order bundled → PATH →
~/.local/bin.  Same contract here; the binary is the C++ `zest` built into zest_amd/_bin.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import time
import urllib.error
import urllib.request
from pathlib import Path

DEFAULT_HTTP_PORT = 9847


def find_binary() -> str:
    """Bundled binary first, then PATH, then ~/.local/bin (reference server.py:78-95)."""
    bundled = Path(__file__).resolve().parent / "_bin" / "zest"
    if bundled.is_file() and os.access(bundled, os.X_OK):
        return str(bundled)
    on_path = shutil.which("zest")
    if on_path:
        return on_path
    local = Path.home() / ".local" / "bin" / "zest"
    if local.is_file():
        return str(local)
    raise FileNotFoundError("zest binary not found (run `python tools/build.py` or put `zest` on PATH)")


def http_port_from_env() -> int:
    try:
        return int(os.environ.get("ZEST_HTTP_PORT", DEFAULT_HTTP_PORT))
    except ValueError:
        return DEFAULT_HTTP_PORT


class ZestServer:
    def __init__(self, http_port: int | None = None, listen_port: int | None = None):
        self.http_port = http_port or http_port_from_env()
        self.listen_port = listen_port
        self.proc: subprocess.Popen | None = None

    @property
    def base_url(self) -> str:
        return f"http://127.0.0.1:{self.http_port}"

    def is_running(self, timeout: float = 1.0) -> bool:
        try:
            with urllib.request.urlopen(self.base_url + "/v1/health", timeout=timeout) as r:
                return r.status == 200
        except (urllib.error.URLError, OSError):
            return False

    def ensure_running(self, wait_s: float = 5.0) -> None:
        if self.is_running():
            return
        cmd = [find_binary(), "serve", "--http-port", str(self.http_port)]
        if self.listen_port:
            cmd += ["--listen-port", str(self.listen_port)]
        # Detached child (new session) so it outlives this interpreter, like `zest start`.
        self.proc = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL,
                                     stderr=subprocess.DEVNULL, start_new_session=True)
        t0 = time.time()
        while time.time() - t0 < wait_s:
            if self.is_running(timeout=0.5):
                return
            if self.proc.poll() is not None:
                raise RuntimeError(f"zest serve exited with code {self.proc.returncode}")
            time.sleep(0.2)
        raise TimeoutError(f"zest server did not become healthy on port {self.http_port}")

    def stop(self, wait_s: float = 5.0) -> bool:
        try:
            req = urllib.request.Request(self.base_url + "/v1/stop", data=b"", method="POST")
            urllib.request.urlopen(req, timeout=2).read()
        except (urllib.error.URLError, OSError):
            return False
        t0 = time.time()
        while time.time() - t0 < wait_s:
            if not self.is_running(timeout=0.3):
                if self.proc is not None:
                    try:
                        self.proc.wait(timeout=wait_s)
                    except subprocess.TimeoutExpired:
                        pass
                return True
            time.sleep(0.1)
        return False

    def status(self) -> dict:
        with urllib.request.urlopen(self.base_url + "/v1/status", timeout=2) as r:
            return json.loads(r.read())
