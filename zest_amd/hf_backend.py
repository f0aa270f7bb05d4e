"""huggingface_hub integration: route snapshot_download / hf_hub_download through zest.

Reference: python/zest/hf_backend.py:1-50 patches only the module attribute
`huggingface_hub.snapshot_download` (so `from huggingface_hub import snapshot_download` done
before enable() is not affected, and `hf_hub_download` is never accelerated).  Here both entry
points are wrapped, in `huggingface_hub` and in the submodules / already-imported consumers
(transformers) that hold their own references; every wrapper falls back to the original function
on any failure, and unpatch restores exactly what was replaced.
"""
from __future__ import annotations

import logging
import os
import sys
import threading
import time
from typing import Any

log = logging.getLogger("zest")
_originals: dict[tuple[str, str], Any] = {}
_client = None
_listings: dict[tuple[str, str, str], tuple[float, frozenset]] = {}
_listings_lock = threading.Lock()
_LISTING_TTL = 30.0


def _repo_paths(repo_id: str, revision: str, repo_type: str) -> frozenset | None:
    """Paths in the repo at `revision` (cached briefly: transformers probes many optional files)."""
    key = (repo_id, revision, repo_type)
    now = time.monotonic()
    with _listings_lock:
        hit = _listings.get(key)
        if hit and now - hit[0] < _LISTING_TTL:
            return hit[1]
    try:
        from . import _core

        _, files = _core.list_repo_files(repo_id, revision, repo_type)
    except Exception:
        return None
    paths = frozenset(f["path"] for f in files)
    with _listings_lock:
        _listings[key] = (now, paths)
    return paths

# (module, attribute) pairs that may hold the functions we wrap.
_SNAPSHOT_SITES = [("huggingface_hub", "snapshot_download"),
                   ("huggingface_hub._snapshot_download", "snapshot_download"),
                   ("transformers.utils.hub", "snapshot_download")]
_FILE_SITES = [("huggingface_hub", "hf_hub_download"),
               ("huggingface_hub.file_download", "hf_hub_download"),
               ("transformers.utils.hub", "hf_hub_download")]


def _unsupported(kwargs: dict) -> bool:
    # Options zest does not implement: let huggingface_hub handle them.
    if kwargs.get("local_dir") or kwargs.get("local_files_only"):
        return True
    rt = kwargs.get("repo_type")
    return rt not in (None, "model", "dataset")


def _wrap_snapshot(orig):
    def zest_snapshot_download(repo_id, *args, revision=None, **kwargs):
        if not args and not _unsupported(kwargs):
            try:
                include = kwargs.get("allow_patterns")
                res = _client.pull_detailed(repo_id, revision or "main", repo_type=kwargs.get("repo_type") or "model",
                                            include=_suffixes(include))
                if res.snapshot_dir and os.path.isdir(res.snapshot_dir):
                    return res.snapshot_dir
            except Exception as e:  # fall back to huggingface_hub
                log.warning("zest: snapshot_download(%s) falling back to huggingface_hub: %s", repo_id, e)
        return orig(repo_id, *args, revision=revision, **kwargs)

    zest_snapshot_download.__wrapped__ = orig
    zest_snapshot_download.__zest__ = True
    return zest_snapshot_download


def _wrap_file(orig):
    def zest_hf_hub_download(repo_id, filename, *args, subfolder=None, revision=None, **kwargs):
        if not args and not _unsupported(kwargs):
            path = f"{subfolder}/{filename}" if subfolder else filename
            rt = kwargs.get("repo_type") or "model"
            paths = _repo_paths(repo_id, revision or "main", rt)
            if paths is not None and path not in paths:
                # transformers probes optional files (adapter_config.json, ...): answer like the Hub does
                from huggingface_hub.errors import EntryNotFoundError

                raise EntryNotFoundError(f"{path} is not in {repo_id}@{revision or 'main'}")
            try:
                res = _client.pull_detailed(repo_id, revision or "main", repo_type=kwargs.get("repo_type") or "model",
                                            include=[path])
                full = os.path.join(res.snapshot_dir, path)
                if os.path.isfile(full):
                    return full
                log.warning("zest: %s missing from snapshot %s; falling back to huggingface_hub", path,
                            res.snapshot_dir)
            except Exception as e:
                log.warning("zest: hf_hub_download(%s, %s) falling back to huggingface_hub: %s", repo_id, path, e)
        return orig(repo_id, filename, *args, subfolder=subfolder, revision=revision, **kwargs)

    zest_hf_hub_download.__wrapped__ = orig
    zest_hf_hub_download.__zest__ = True
    return zest_hf_hub_download


def _suffixes(patterns) -> list[str] | None:
    """allow_patterns → suffix filters understood by the native pull (only plain '*.ext' / names)."""
    if not patterns:
        return None
    if isinstance(patterns, str):
        patterns = [patterns]
    out = []
    for p in patterns:
        if p.startswith("*") and not any(c in p[1:] for c in "*?["):
            out.append(p[1:])
        elif not any(c in p for c in "*?["):
            out.append(p)
        else:
            raise ValueError("pattern not supported natively")  # caller falls back
    return out


def patch_hf_hub(client) -> bool:
    """Install the wrappers; returns False when huggingface_hub is not importable."""
    global _client
    try:
        import huggingface_hub  # noqa: F401
    except ImportError:
        return False
    _client = client
    for sites, wrap in ((_SNAPSHOT_SITES, _wrap_snapshot), (_FILE_SITES, _wrap_file)):
        for mod_name, attr in sites:
            mod = sys.modules.get(mod_name)
            if mod is None and mod_name.startswith("huggingface_hub"):
                try:
                    __import__(mod_name)
                    mod = sys.modules.get(mod_name)
                except ImportError:
                    mod = None
            if mod is None or not hasattr(mod, attr):
                continue
            cur = getattr(mod, attr)
            if getattr(cur, "__zest__", False):
                continue
            _originals[(mod_name, attr)] = cur
            setattr(mod, attr, wrap(cur))
    return True


def unpatch_hf_hub() -> None:
    for (mod_name, attr), orig in list(_originals.items()):
        mod = sys.modules.get(mod_name)
        if mod is not None:
            setattr(mod, attr, orig)
    _originals.clear()


def is_patched() -> bool:
    return bool(_originals)
