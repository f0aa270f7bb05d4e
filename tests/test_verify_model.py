"""End-to-end model check (the reference's test/local/verify-model.sh, offline): a GPT-2 checkpoint
is published on the fake Hub, pulled with `zest pull` and with `zest.enable()` +
`AutoModelForCausalLM.from_pretrained(repo_id)`, loaded with transformers and run.  Its logits
and greedy continuation must match the model that was uploaded.

The reference pulls openai-community/gpt2 from the real Hub; without network the checkpoint is a
randomly initialised GPT-2 with a small config, saved by transformers itself (safetensors)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from e2e_util import Node, free_port
from zest_amd.testing import FakeHub

transformers = pytest.importorskip("transformers")

REPO = "openai-community/gpt2-zest-test"
ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def gpt2_checkpoint(tmp_path_factory):
    torch.manual_seed(0)
    cfg = transformers.GPT2Config(n_layer=2, n_head=4, n_embd=128, vocab_size=2048, n_positions=128)
    model = transformers.GPT2LMHeadModel(cfg).eval()
    d = tmp_path_factory.mktemp("gpt2")
    model.save_pretrained(d, safe_serialization=True)
    files = {p.name: p.read_bytes() for p in d.iterdir() if p.is_file()}
    assert "model.safetensors" in files and "config.json" in files
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    with torch.no_grad():
        logits = model(ids).logits
        gen = model.generate(ids[:1], max_new_tokens=8, do_sample=False, pad_token_id=0)
    return files, ids, logits, gen


@pytest.fixture
def hub_with_gpt2(gpt2_checkpoint):
    files = gpt2_checkpoint[0]
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    commit = hub.add_repo(REPO, files, xet_min_size=100_000)
    yield hub, commit
    hub.stop()


def _check(model_dir_or_id, gpt2_checkpoint):
    _, ids, logits, gen = gpt2_checkpoint
    model = transformers.AutoModelForCausalLM.from_pretrained(model_dir_or_id, torch_dtype=torch.float32).eval()
    assert sum(p.numel() for p in model.parameters()) > 300_000
    with torch.no_grad():
        assert torch.equal(model(ids).logits, logits)
        assert torch.equal(model.generate(ids[:1], max_new_tokens=8, do_sample=False, pad_token_id=0), gen)


def test_cli_pull_then_transformers_inference(hub_with_gpt2, gpt2_checkpoint, tmp_path):
    hub, commit = hub_with_gpt2
    node = Node(hub, tmp_path, "verify")
    try:
        out = node.run("pull", REPO, "--no-p2p").stdout
        assert "Done!" in out
        snap = node.snapshot(REPO, commit)
        assert (snap / "model.safetensors").is_file()
        _check(str(snap), gpt2_checkpoint)
    finally:
        node.close()


_ENABLE_SCRIPT = r"""
import os, sys, torch
import zest_amd as zest
zest.enable()                                   # before transformers is imported, like a user script
from transformers import AutoModelForCausalLM
ids, logits, gen = torch.load(sys.argv[1], weights_only=True)
m = AutoModelForCausalLM.from_pretrained(sys.argv[2], torch_dtype=torch.float32).eval()
with torch.no_grad():
    assert torch.equal(m(ids).logits, logits)
    assert torch.equal(m.generate(ids[:1], max_new_tokens=8, do_sample=False, pad_token_id=0), gen)
st = zest.status()
zest.disable()
zest.stop()
print("OK", st.get("version"))
"""


def test_enable_from_pretrained_repo_id(hub_with_gpt2, gpt2_checkpoint, tmp_path):
    """`import zest; zest.enable(); AutoModelForCausalLM.from_pretrained(repo)`, in a
    fresh interpreter so huggingface_hub reads HF_ENDPOINT / HF_HUB_CACHE from this environment."""
    hub, commit = hub_with_gpt2
    _, ids, logits, gen = gpt2_checkpoint
    ref = tmp_path / "ref.pt"
    torch.save((ids, logits, gen), ref)
    env = dict(os.environ, **hub.env(str(tmp_path)), ZEST_HTTP_PORT=str(free_port()),
               ZEST_LISTEN_PORT=str(free_port()), PYTHONPATH=str(ROOT))
    env.pop("ZEST_NO_AUTOSTART")
    for k in ("HF_HUB_OFFLINE", "TRANSFORMERS_OFFLINE"):  # the "Hub" is the local fake
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _ENABLE_SCRIPT, str(ref), REPO], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    snap = tmp_path / "hf" / "hub" / ("models--" + REPO.replace("/", "--")) / "snapshots" / commit
    assert (snap / "model.safetensors").is_file()
    assert "falling back to huggingface_hub" not in r.stderr, r.stderr[-4000:]  # zest served every file
    assert hub.counters.get("xorb_get", 0) > 0


def _zest_from_pretrained(hub, tmp_path, monkeypatch, device, direct):
    import zest_amd

    for k, v in hub.env(str(tmp_path)).items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
    return zest_amd.from_pretrained(REPO, device=device, direct=direct, p2p=False, dht=False)


def test_zest_from_pretrained_cpu(hub_with_gpt2, gpt2_checkpoint, tmp_path, monkeypatch):
    """zest_amd.from_pretrained: the model is built around the pulled, hash-verified tensors (no
    second copy); logits and greedy generation match the uploaded model."""
    hub, commit = hub_with_gpt2
    _, ids, logits, gen = gpt2_checkpoint
    model = _zest_from_pretrained(hub, tmp_path, monkeypatch, "cpu", False)
    assert type(model).__name__ == "GPT2LMHeadModel"
    assert all(p.device.type == "cpu" for p in model.parameters())
    with torch.no_grad():
        assert torch.equal(model(ids).logits, logits)
        assert torch.equal(model.generate(ids[:1], max_new_tokens=8, do_sample=False, pad_token_id=0), gen)
    # config/tokenizer files are in the snapshot; the weights never went through from_pretrained's reader
    assert (Path(model.zest_snapshot_dir) / "config.json").is_file()


@pytest.mark.gpu
def test_zest_from_pretrained_direct_to_hbm(hub_with_gpt2, gpt2_checkpoint, tmp_path, monkeypatch):
    """Network -> HBM (GPU decode + Merkle verify, no disk for the weights) -> transformers model whose
    parameters are those HBM buffers; outputs match the uploaded model."""
    hub, commit = hub_with_gpt2
    files, ids, logits, gen = gpt2_checkpoint
    model = _zest_from_pretrained(hub, tmp_path, monkeypatch, "cuda:0", True)
    assert all(p.device.type == "cuda" for p in model.parameters())
    snap = Path(model.zest_snapshot_dir)
    assert not (snap / "model.safetensors").exists()  # weights bypassed the disk
    import safetensors.torch as st

    want = st.load(files["model.safetensors"])
    got = model.state_dict()
    for k, v in want.items():
        assert torch.equal(got[k].cpu(), v), k
    with torch.no_grad():
        out = model(ids.cuda()).logits.cpu()
    assert torch.allclose(out, logits, atol=1e-4, rtol=1e-4)


def _fp_all_worker(rank, world, port, env, ref, q):
    import torch.distributed as dist

    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import zest_amd
        ids, logits, gen = torch.load(ref, weights_only=True)
        m = zest_amd.from_pretrained(REPO, device="all", p2p=False, dht=False)
        with torch.no_grad():
            ok = torch.equal(m(ids).logits, logits) and torch.equal(
                m.generate(ids[:1], max_new_tokens=8, do_sample=False, pad_token_id=0), gen)
        q.put((rank, ok, ""))
    except Exception as e:  # reported to the parent
        q.put((rank, False, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def test_zest_from_pretrained_all_ranks(hub_with_gpt2, gpt2_checkpoint, tmp_path):
    """from_pretrained(device="all") on a 2-rank CPU process group: the weights come from the swarm
    pull (each file fetched by one rank, broadcast to the other, re-verified), every rank gets a
    working model with the uploaded model's logits and generation."""
    import torch.multiprocessing as mp

    hub, commit = hub_with_gpt2
    _, ids, logits, gen = gpt2_checkpoint
    ref = tmp_path / "ref.pt"
    torch.save((ids, logits, gen), ref)
    env = dict(hub.env(str(tmp_path)), ZEST_LISTEN_PORT=str(free_port()))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_fp_all_worker, args=(r, 2, port, env, str(ref), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
