"""zest_amd — MI355X-native P2P model distribution (zest capabilities, rebuilt for AMD CDNA4).

Usage (same API as the reference's `zest` package, python/zest/__init__.py:1-73):

    import zest_amd as zest          # or: import zest  (compat shim)
    zest.enable()                    # background seeder + huggingface_hub patch
    path = zest.pull("meta-llama/Llama-3.1-8B")
    weights = zest.pull("meta-llama/Llama-3.1-8B", device="cuda:0")   # HBM tensors, GPU-verified
    model = zest.from_pretrained("meta-llama/Llama-3.1-8B")            # transformers model on those tensors
    print(zest.status()); zest.stop()

Layers (see docs/ARCHITECTURE.md):
  zest_amd._core    C++17 host core: BLAKE3/Xet hashing, LZ4/BG4, CDC, xorbs, BT/DHT/HTTP stack
  zest_amd._hip     HIP/CDNA4 kernels for gfx950: xorb ingest (decode+verify), BLAKE3, Merkle, CDC
  zest_amd.ops      torch-facing wrappers of the HIP kernels
  zest_amd.parallel RCCL (torch.distributed "nccl") intra-node swarm: GPUs as BitTorrent peers
  zest_amd.models   synthetic model specs (gpt2, Llama-3.1-8B/70B, Qwen2-7B, Mixtral-8x7B)
  zest_amd.utils    tracing, fault-injection spec, formatting helpers
"""
from __future__ import annotations

import os

__version__ = "0.4.2"

_server = None
_client = None


def _init():
    global _server, _client
    if _server is None:
        from .client import ZestClient
        from .server import ZestServer

        _server = ZestServer()
        _client = ZestClient()


def enable() -> None:
    """Start the background zest server (seeding) and route huggingface_hub downloads through zest."""
    _init()
    _server.ensure_running()
    from .hf_backend import patch_hf_hub

    patch_hf_hub(_client)


def disable() -> None:
    """Restore the original huggingface_hub functions."""
    from .hf_backend import unpatch_hf_hub

    unpatch_hf_hub()


def pull(repo: str, revision: str = "main", *, device=None, as_tensors: bool = False, verify: bool = True,
         p2p: bool = True, peers=None, tracker=None, dht: bool = True, dht_bootstrap=None, include=None,
         group=None, repo_type: str = "model", verbose: bool = False, direct: bool | None = None,
         save_snapshot: bool = False, threads: int = 16, staging_bytes: int = 1 << 30, stats: dict | None = None,
         exchange: str = "auto", round_bytes: int | None = None):
    """Download `repo@revision` via zest.

    * default: returns the HF-cache snapshot directory (reference behaviour).
    * device="cuda:N" (or as_tensors=True): also loads every *.safetensors file into that GPU's HBM,
      verifies each against its Xet file hash on the GPU, and returns {tensor_name: tensor}.
    * device="all": collective over `group` (default WORLD) — every rank gets all tensors on its
      own GPU (CPU process groups: host memory).  The model's reconstruction terms are split into
      byte-balanced per-rank shares; each rank fetches its share device-direct, round by round,
      and the rounds are replicated over xGMI with the exchange strategy measured fastest at setup
      (`exchange`, default "auto"), every received chunk re-hashed on the receiver, every file
      Merkle-checked on every rank; no snapshot is written (zest_amd.parallel.swarm_pull).
      `stats` (a dict) receives the exchange mode used, bytes fetched / received, per-phase
      seconds, re-shards and recovered ranks.
    * device="cuda:N" / "cpu" pulls are device-direct by default (`direct=None` -> True, like
      from_pretrained): Xet files bypass the disk -- fetched compressed through the
      cache/peer/CDN waterfall and decoded + hash-verified on the GPU into HBM (zest_amd.direct);
      `threads` fetch workers fill pinned staging buffers of `staging_bytes` each.  With
      device="cpu" the same pull lands in CPU tensors (host decode + verification, no disk).  No
      snapshot is written unless `save_snapshot=True`; `include` (file-name suffixes) filters the
      safetensors files.  direct=False: the reference's path -- the CLI writes the HF-cache
      snapshot, which is then loaded and (verify=True) hash-checked on the device.
    """
    _init()
    kw = dict(p2p=p2p, peers=peers, tracker=tracker, dht=dht, dht_bootstrap=dht_bootstrap, include=include,
              verify=verify, repo_type=repo_type, verbose=verbose)
    if device is None and not as_tensors:
        return _client.pull(repo, revision, **kw)
    if device == "all":
        from .parallel import swarm_pull

        return swarm_pull(repo, revision, group=group, p2p=p2p, peers=peers, tracker=tracker, dht=dht,
                          dht_bootstrap=dht_bootstrap, repo_type=repo_type, verify_received=verify,
                          staging_bytes=staging_bytes, threads=threads, stats=stats, exchange=exchange,
                          round_bytes=round_bytes)
    if direct is None:
        direct = True  # weights straight into device memory (the north star); direct=False: via disk
    if direct:
        from .direct import pull_to_device

        return pull_to_device(repo, revision, device or "cuda:0", p2p=p2p, peers=peers, tracker=tracker, dht=dht,
                              dht_bootstrap=dht_bootstrap, repo_type=repo_type, save_snapshot=save_snapshot,
                              threads=threads, staging_bytes=staging_bytes, include=include)
    from .device import load_snapshot

    res = _client.pull_detailed(repo, revision, **kw)
    return load_snapshot(res.snapshot_dir, device or "cuda:0", res.xet_hashes() if verify else None)


def from_pretrained(repo: str, revision: str = "main", **kw):
    """transformers model built around weights pulled into `device` memory (zest_amd.hf_model)."""
    from .hf_model import from_pretrained as _fp

    return _fp(repo, revision, **kw)


def status() -> dict:
    """Status JSON of the background server (starting it if needed)."""
    _init()
    _server.ensure_running()
    return _client.status()


def stop() -> None:
    """Stop the background server."""
    _init()
    _server.stop()


# Auto-enable when ZEST=1 is set (reference python/zest/__init__.py:68-73).
if os.environ.get("ZEST", "").strip().lower() in ("1", "true", "yes"):
    try:
        enable()
    except Exception:
        pass
