"""Device-direct pull: Xet files go from the network (peers / CDN / local xorb cache) to HBM with
GPU-side decode and verification (`_hip.DeviceXetPull`); the host only moves compressed bytes.

    tensors = pull_to_device("meta-llama/Llama-3.1-8B", device="cuda:0")
    tensors = pull_to_device("meta-llama/Llama-3.1-8B", device="cpu")   # in memory, no disk

device="cpu": the same fetch through the host waterfall straight into CPU tensors
(`_core.HostXetFetcher`: CPU decode + BLAKE3/Merkle verification, no snapshot written).

Non-Xet files of the repo (config, tokenizer, small safetensors) are fetched by the native host
pull (`include=` filter) and loaded like the disk path.  With `save_snapshot=True` the verified
device bytes are also written to the HF cache snapshot so later `from_pretrained` calls hit disk.
"""
from __future__ import annotations

import os
import struct

import torch

from . import _core, ops
from . import device as zdev


def pull_to_device(repo: str, revision: str = "main", device="cuda:0", *, p2p: bool = True, peers=None,
                   tracker=None, dht: bool = True, dht_bootstrap=None, repo_type: str = "model",
                   save_snapshot: bool = False, staging_bytes: int = 1 << 30, threads: int = 16, include=None):
    dev = torch.device(device)
    if dev.type not in ("cuda", "cpu"):
        raise ValueError("pull_to_device needs a GPU or the CPU")
    commit, files = _core.list_repo_files(repo, revision, repo_type)
    if include:  # file-name suffixes, as `zest pull --include` (csrc/core/pull.cpp)
        files = [f for f in files if any(f["path"].endswith(x) for x in include)]
    st_files = [f for f in files if f["path"].endswith(".safetensors")]
    xet = [f for f in st_files if f["xet_hash"]]
    plain = [f for f in st_files if not f["xet_hash"]]
    out: dict[str, torch.Tensor] = {}
    if xet and dev.type == "cpu":
        hf = _core.HostXetFetcher(repo, revision, repo_type, p2p, list(peers or []), tracker, dht,
                                  list(dht_bootstrap or []), threads)
        bufs = [torch.empty(f["size"], dtype=torch.uint8) for f in xet]
        hf.fetch_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in zip(xet, bufs)])
        for f, buf in zip(xet, bufs):
            _add_views(out, buf, f["path"])
            if save_snapshot:
                _save(repo, commit or revision, f["path"], buf)
    elif xet:
        dp = ops.hip().DeviceXetPull(repo, revision, repo_type, p2p, list(peers or []), tracker, dht,
                                     list(dht_bootstrap or []), dev.index or 0, staging_bytes, threads)
        bufs = [ops.padded_empty(f["size"], dev)[:f["size"]] for f in xet]
        torch.cuda.synchronize(dev)  # allocations visible to the pull's private stream
        # one pipeline for all files: staging batches cross file boundaries
        dp.pull_files([(f["xet_hash"], b.data_ptr(), f["size"]) for f, b in zip(xet, bufs)])
        for f, buf in zip(xet, bufs):
            _add_views(out, buf, f["path"])
            if save_snapshot:
                _save(repo, commit or revision, f["path"], buf)
    if plain or save_snapshot:
        inc = [f["path"] for f in plain] + ([f["path"] for f in files if not f["path"].endswith(".safetensors")]
                                           if save_snapshot else [])
        if inc:
            r = _core.pull(repo, revision, p2p, list(peers or []), tracker, dht, list(dht_bootstrap or []), inc,
                           True, 0, repo_type)
            for f in plain:
                buf = zdev.load_file(os.path.join(r["snapshot_dir"], f["path"]), dev)
                _add_views(out, buf, f["path"])
    return out


def _add_views(out: dict, buf: torch.Tensor, path: str) -> None:
    (hlen,) = struct.unpack("<Q", buf[:8].cpu().numpy().tobytes())
    start, meta = zdev.parse_safetensors_header(buf[:8 + hlen].cpu().numpy().tobytes())
    for k, v in zdev.tensor_views(buf, start, meta).items():
        if k in out:
            raise ValueError(f"duplicate tensor {k} in {path}")
        out[k] = v


def _save(repo: str, commit: str, path: str, buf: torch.Tensor) -> None:
    import json

    cfg = json.loads(_core.config_json())
    snap = os.path.join(cfg["hf_cache_dir"], _core.repo_folder_name(repo), "snapshots", commit)
    dst = os.path.join(snap, path)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    tmp = dst + ".incomplete"
    buf.cpu().numpy().tofile(tmp)
    os.replace(tmp, dst)
