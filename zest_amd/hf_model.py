"""`from_pretrained` on weights that are already resident: pull a repository's safetensors into GPU
memory (GPU-verified against their Xet hashes, optionally network -> HBM with no disk at all) and
build the transformers model around those tensors without copying them.

    model = zest_amd.from_pretrained("meta-llama/Llama-3.1-8B", device="cuda:0")

The reference stops at files in the HF cache that `from_pretrained` then reads and copies again
(python/zest/hf_backend.py:9-33, examples/download_model.py:1-31); here the parameters ARE the
pulled buffers: transformers assigns the state dict into a meta-initialised model (no random init,
no second copy), so peak device memory is one model.  Config / tokenizer / other small files come
through the native host pull into the HF snapshot, so `AutoTokenizer.from_pretrained(snapshot)`
works as usual.
"""
from __future__ import annotations

from . import _core


def snapshot_without_weights(repo: str, revision: str = "main", *, p2p: bool = True, peers=None, tracker=None,
                             dht: bool = True, dht_bootstrap=None, repo_type: str = "model") -> str:
    """Pull every non-safetensors file (config, tokenizer, ...) into the HF snapshot; returns its dir."""
    _commit, files = _core.list_repo_files(repo, revision, repo_type)
    other = [f["path"] for f in files if not f["path"].endswith(".safetensors")]
    if not other:
        raise FileNotFoundError(f"{repo}@{revision}: no config files to build a model from")
    r = _core.pull(repo, revision, p2p, list(peers or []), tracker, dht, list(dht_bootstrap or []), other, True, 0,
                   repo_type)
    if r["failed_files"]:
        raise RuntimeError(f"{repo}@{revision}: {r['failed_files']} file(s) failed")
    return r["snapshot_dir"]


def model_class(config, auto_class="AutoModelForCausalLM"):
    """Concrete transformers class for `config` under an Auto class (name or class)."""
    import transformers

    auto = getattr(transformers, auto_class) if isinstance(auto_class, str) else auto_class
    return auto._model_mapping[type(config)]


def from_pretrained(repo: str, revision: str = "main", *, device="cuda:0", direct: bool = True,
                    auto_class="AutoModelForCausalLM", p2p: bool = True, peers=None, tracker=None, dht: bool = True,
                    dht_bootstrap=None, repo_type: str = "model", verify: bool = True, group=None, **model_kwargs):
    """A transformers model whose parameters are zest-pulled, hash-verified tensors on `device`.

    direct=True (GPU only): Xet files go network -> pinned staging -> HBM with GPU decode + Merkle
    verification and never touch the disk; otherwise the files land in the HF cache first and are
    streamed to `device` and verified there.  device="all": collective over `group` (one process per
    GPU): the weights come from the intra-node swarm pull (each file fetched once by one rank,
    seeded to the others over xGMI, re-verified everywhere) and every rank gets a model on its own
    device; rank 0 alone fetches the config / tokenizer files.  Extra keyword arguments go to the
    model class's `from_pretrained` (e.g. attn_implementation); a `dtype` different from the
    checkpoint's makes transformers convert (copy) the weights.
    """
    import torch
    import transformers

    from . import pull

    if device == "all":
        import torch.distributed as dist

        obj = [None]
        if dist.get_rank(group) == 0:
            try:
                obj[0] = ("ok", snapshot_without_weights(repo, revision, p2p=p2p, peers=peers, tracker=tracker,
                                                         dht=dht, dht_bootstrap=dht_bootstrap, repo_type=repo_type))
            except Exception as e:  # every rank leaves the same way
                obj[0] = ("err", f"{type(e).__name__}: {e}")
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if obj[0][0] != "ok":
            raise RuntimeError(f"{repo}@{revision}: config files: {obj[0][1]}")
        snap = obj[0][1]
        weights = pull(repo, revision, device="all", group=group, verify=verify, p2p=p2p, peers=peers,
                       tracker=tracker, dht=dht, dht_bootstrap=dht_bootstrap, repo_type=repo_type)
        dev = next(iter(weights.values())).device if weights else torch.device("cpu")
        config = transformers.AutoConfig.from_pretrained(snap)
    else:
        dev = torch.device(device)
        snap = snapshot_without_weights(repo, revision, p2p=p2p, peers=peers, tracker=tracker, dht=dht,
                                        dht_bootstrap=dht_bootstrap, repo_type=repo_type)
        config = transformers.AutoConfig.from_pretrained(snap)
        weights = pull(repo, revision, device=dev, direct=direct and dev.type == "cuda", verify=verify, p2p=p2p,
                       peers=peers, tracker=tracker, dht=dht, dht_bootstrap=dht_bootstrap, repo_type=repo_type)
    cls = model_class(config, auto_class)
    # place the model where the weights already are (without a device_map transformers would
    # materialise it on the CPU and copy the tensors there)
    model_kwargs.setdefault("device_map", {"": str(dev)})
    model = cls.from_pretrained(None, config=config, state_dict=weights, **model_kwargs)
    model.eval()
    model.zest_snapshot_dir = snap  # where the tokenizer / generation config live
    return model
