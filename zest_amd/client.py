"""Client side of `zest.pull`: runs the native pull in-process and returns the snapshot path.

Reference: python/zest/client.py:1-71 shells out to `zest pull` and then guesses the snapshot as
the most recently modified directory under ~/.cache/huggingface/hub (ignoring HF_HOME).  Here the
native pull (`_core.pull`, C++: hub listing → CAS reconstruction → cache/P2P/CDN waterfall →
verified HF-layout snapshot) runs in-process with the GIL released and reports the exact snapshot
directory it wrote, honouring HF_HUB_CACHE / HF_HOME.
"""
from __future__ import annotations

import json
import urllib.request
from dataclasses import dataclass, field

from . import _core
from .server import http_port_from_env


class PullError(RuntimeError):
    pass


@dataclass
class PullResult:
    snapshot_dir: str
    commit: str
    files: int
    xet_files: int
    cached_files: int
    bytes: int
    bytes_from_peer: int
    bytes_from_cdn: int
    bytes_from_cache: int
    seconds: float
    log: str = ""
    stats: dict = field(default_factory=dict)
    file_list: list = field(default_factory=list)  # [{"path","size","xet_hash","ok"}]

    def xet_hashes(self) -> dict[str, str]:
        return {f["path"]: f["xet_hash"] for f in self.file_list if f.get("xet_hash")}

    @property
    def p2p_ratio(self) -> float:
        tot = self.bytes_from_peer + self.bytes_from_cdn + self.bytes_from_cache
        return self.bytes_from_peer / tot if tot else 0.0


class ZestClient:
    def __init__(self, http_port: int | None = None):
        self.http_port = http_port or http_port_from_env()

    def pull_detailed(self, repo: str, revision: str = "main", *, p2p: bool = True, peers=None, tracker=None,
                      dht: bool = True, dht_bootstrap=None, include=None, verify: bool = True,
                      concurrency: int = 0, repo_type: str = "model", verbose: bool = False) -> PullResult:
        r = _core.pull(repo, revision, p2p, list(peers or []), tracker, dht, list(dht_bootstrap or []),
                       list(include or []), verify, concurrency, repo_type)
        if verbose:
            print(r["stdout"], end="")
        if r["failed_files"]:
            raise PullError(f"pull {repo}@{revision}: {r['failed_files']} file(s) failed:\n{r['stderr']}")
        return PullResult(r["snapshot_dir"], r["commit"], r["files"], r["xet_files"], r["cached_files"], r["bytes"],
                          r["bytes_from_peer"], r["bytes_from_cdn"], r["bytes_from_cache"], r["seconds"],
                          r["stdout"] + r["stderr"], json.loads(r["stats_json"] or "{}"),
                          json.loads(r["files_json"] or "[]"))

    def pull(self, repo: str, revision: str = "main", **kw) -> str:
        return self.pull_detailed(repo, revision, **kw).snapshot_dir

    def status(self) -> dict:
        with urllib.request.urlopen(f"http://127.0.0.1:{self.http_port}/v1/status", timeout=2) as r:
            return json.loads(r.read())
