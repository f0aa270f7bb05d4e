"""Python API: zest_amd.pull / enable / disable / status / stop, huggingface_hub patching,
device tensor loading (CPU path here; the GPU path is in test_gpu_device.py) and the swarm load
over a gloo process group."""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest
import torch

from e2e_util import free_port
import zest_amd
import zest_amd.client  # noqa: F401  (submodule used as zest_amd.client below)
from zest_amd import device as zdev
from zest_amd import hf_backend, models
from zest_amd.synthetic import SyntheticWorld
from zest_amd.testing import FakeHub


@pytest.fixture
def world_hub(tmp_path, monkeypatch):
    world = SyntheticWorld(models.get("llama-tiny"), seed=7, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=1 << 20)
    hub.start()
    commit = hub.add_world(world)
    for k, v in hub.env(str(tmp_path)).items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("ZEST_HTTP_PORT", str(free_port()))
    monkeypatch.setenv("ZEST_LISTEN_PORT", str(free_port()))
    yield world, hub, commit
    hub.stop()


def _expected_tensors(world):
    out = {}
    for f in world.xet_files:
        data = world.file_bytes_host(f)
        (hlen,) = struct.unpack("<Q", data[:8])
        meta = json.loads(data[8:8 + hlen])
        for name, ent in meta.items():
            if name == "__metadata__":
                continue
            a, b = ent["data_offsets"]
            out[name] = (ent["dtype"], ent["shape"], data[8 + hlen + a:8 + hlen + b])
    return out


def test_pull_returns_snapshot(world_hub):
    world, hub, commit = world_hub
    path = zest_amd.pull(world.spec.repo_id, p2p=False)
    assert path.endswith(f"/snapshots/{commit}")
    for f in world.files:
        with open(os.path.join(path, f.path), "rb") as fh:
            assert fh.read() == world.file_bytes_host(f)


def test_pull_as_tensors_cpu(world_hub):
    world, hub, commit = world_hub
    tensors = zest_amd.pull(world.spec.repo_id, device="cpu", p2p=False)
    exp = _expected_tensors(world)
    assert set(tensors) == set(exp)
    for name, (dt, shape, raw) in exp.items():
        t = tensors[name]
        assert list(t.shape) == shape and t.dtype == zdev.ST_DTYPES[dt]
        assert t.contiguous().view(torch.uint8).numpy().tobytes() == raw


def test_pull_device_defaults_to_direct(world_hub, tmp_path):
    """A device pull is device-direct by default (as from_pretrained): tensors straight into device
    memory, no snapshot on disk unless save_snapshot=True; direct=False is the snapshot path;
    include (suffixes) filters the files."""
    import inspect

    world, hub, commit = world_hub
    assert inspect.signature(zest_amd.pull).parameters["direct"].default is None
    hf = tmp_path / "hf"

    def snaps():
        return sorted(p.name for p in hf.rglob("*.safetensors")) if hf.exists() else []
    exp = _expected_tensors(world)
    got = zest_amd.pull(world.spec.repo_id, device="cpu", p2p=False, dht=False)
    assert set(got) == set(exp) and snaps() == []
    one = world.xet_files[0].path
    part = zest_amd.pull(world.spec.repo_id, device="cpu", p2p=False, dht=False, include=[one])
    assert part and set(part) <= set(exp)
    assert zest_amd.pull(world.spec.repo_id, device="cpu", p2p=False, dht=False, include=["no-such.bin"]) == {}
    got = zest_amd.pull(world.spec.repo_id, device="cpu", p2p=False, dht=False, save_snapshot=True)
    assert set(got) == set(exp) and snaps() == sorted(os.path.basename(f.path) for f in world.files
                                                        if f.path.endswith(".safetensors"))
    legacy = zest_amd.pull(world.spec.repo_id, device="cpu", direct=False, p2p=False)
    assert set(legacy) == set(exp)


def test_load_snapshot_detects_corruption(world_hub):
    world, hub, commit = world_hub
    client = zest_amd.client.ZestClient()
    res = client.pull_detailed(world.spec.repo_id, p2p=False)
    hashes = res.xet_hashes()
    assert set(hashes) == {f.path for f in world.xet_files}
    zdev.load_snapshot(res.snapshot_dir, "cpu", hashes)  # clean: passes
    victim = os.path.join(res.snapshot_dir, world.xet_files[0].path)
    with open(victim, "r+b") as fh:
        fh.seek(os.path.getsize(victim) // 2)
        b = fh.read(1)
        fh.seek(-1, 1)
        fh.write(bytes([b[0] ^ 1]))
    with pytest.raises(zdev.VerifyError):
        zdev.load_snapshot(res.snapshot_dir, "cpu", hashes)


def test_hf_hub_patch(world_hub):
    world, hub, commit = world_hub
    import huggingface_hub

    orig_snap, orig_file = huggingface_hub.snapshot_download, huggingface_hub.hf_hub_download
    client = zest_amd.client.ZestClient()
    assert hf_backend.patch_hf_hub(client)
    try:
        assert huggingface_hub.snapshot_download is not orig_snap
        p = huggingface_hub.snapshot_download(world.spec.repo_id)
        assert p.endswith(commit) and os.path.isfile(os.path.join(p, "config.json"))
        f = huggingface_hub.hf_hub_download(world.spec.repo_id, "config.json")
        assert f.endswith("config.json") and json.load(open(f))
        from huggingface_hub import file_download
        assert getattr(file_download.hf_hub_download, "__zest__", False)
    finally:
        hf_backend.unpatch_hf_hub()
    assert huggingface_hub.snapshot_download is orig_snap
    assert huggingface_hub.hf_hub_download is orig_file
    assert not hf_backend.is_patched()


def test_server_lifecycle_and_status(world_hub):
    zest_amd._server = None
    zest_amd._client = None
    st = zest_amd.status()  # starts the server
    assert st["version"] == zest_amd.__version__
    assert st["http_port"] == int(os.environ["ZEST_HTTP_PORT"])
    zest_amd.stop()
    assert not zest_amd._server.is_running(timeout=0.3)


def test_enable_disable(world_hub):
    import huggingface_hub

    zest_amd._server = None
    zest_amd._client = None
    orig = huggingface_hub.snapshot_download
    zest_amd.enable()
    try:
        assert huggingface_hub.snapshot_download is not orig
    finally:
        zest_amd.disable()
        zest_amd.stop()
    assert huggingface_hub.snapshot_download is orig


def test_cli_module():
    r = subprocess.run([sys.executable, "-m", "zest", "version"], capture_output=True, text=True,
                       cwd=os.path.dirname(os.path.dirname(__file__)))
    assert r.returncode == 0 and r.stdout.strip() == f"zest {zest_amd.__version__}"


def test_assign_owners_balanced():
    from zest_amd.parallel import assign_owners

    sizes = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    own = assign_owners(sizes, 3)
    loads = [sum(s for s, o in zip(sizes, own) if o == r) for r in range(3)]
    assert max(loads) - min(loads) <= 2
    assert assign_owners(sizes, 3) == own  # deterministic


def _swarm_worker(rank, world, port, snap, hashes, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from zest_amd.parallel import swarm_load

        try:
            t = swarm_load(snap, xet_hashes=hashes, verify_all=True)
        except Exception as e:  # noqa: BLE001 - reported to the test
            q.put((rank, type(e).__name__))
            return
        digest = {k: v.contiguous().view(torch.uint8).sum().item() for k, v in t.items()}
        q.put((rank, digest))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_swarm_load_gloo(world_hub, tmp_path, corrupt):
    import torch.multiprocessing as mp

    world, hub, commit = world_hub
    # two shards so both ranks own a file
    spec = models.get("llama-tiny")
    res = zest_amd.client.ZestClient().pull_detailed(world.spec.repo_id, p2p=False)
    # split the single shard into 2 files to exercise multi-owner logic
    src = os.path.join(res.snapshot_dir, world.xet_files[0].path)
    ref = zdev.load_snapshot(res.snapshot_dir, "cpu")
    snap2 = tmp_path / "snap2"
    snap2.mkdir()
    names = sorted(ref)
    half = len(names) // 2
    from zest_amd.models import TensorSpec, safetensors_header

    for part, sel in (("a.safetensors", names[:half]), ("b.safetensors", names[half:])):
        specs = [TensorSpec(n, {torch.bfloat16: "BF16", torch.float32: "F32"}[ref[n].dtype], tuple(ref[n].shape)) for n in sel]
        head, offs = safetensors_header(specs)
        body = b"".join(ref[n].contiguous().view(torch.uint8).numpy().tobytes() for n in sel)
        (snap2 / part).write_bytes(head + body)
    hashes = {p: _core_hash(snap2 / p) for p in ("a.safetensors", "b.safetensors")}
    if corrupt:  # one owner's file fails its hash check: every rank raises, none hangs in a broadcast
        hashes["b.safetensors"] = "0" * 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_swarm_worker, args=(r, 2, port, str(snap2), hashes, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if corrupt:
        assert got == {0: "VerifyError", 1: "VerifyError"}
        return
    exp = {k: v.contiguous().view(torch.uint8).sum().item() for k, v in ref.items()}
    assert got[0] == exp and got[1] == exp
    del spec, src


def _core_hash(path):
    from zest_amd import _core

    return _core.xet_hex(bytes(_core.xet_file_hash(np.fromfile(path, dtype=np.uint8))))


def test_direct_pull_to_cpu_memory(tmp_path, monkeypatch):
    """zest_amd.pull(repo, device="cpu", direct=True): Xet safetensors reconstructed through the host
    waterfall straight into CPU tensors (HostXetFetcher: decode + BLAKE3/Merkle verify), no snapshot;
    tensors equal the uploaded ones."""
    import dataclasses
    import json
    import struct

    import zest_amd
    from zest_amd import models
    from zest_amd.synthetic import SyntheticWorld
    from zest_amd.testing import FakeHub

    spec = dataclasses.replace(models.get("llama-tiny"), max_shard_bytes=700_000)
    world = SyntheticWorld(spec, seed=4, mode="bf16")
    hub = FakeHub(policy="auto", max_xorb_bytes=256 << 10)
    hub.start()
    try:
        hub.add_world(world)
        for k, v in hub.env(str(tmp_path)).items():
            monkeypatch.setenv(k, v)
        got = zest_amd.pull(spec.repo_id, device="cpu", direct=True, p2p=False, dht=False)
        want = {}
        for f in world.xet_files:
            data = world.file_bytes_host(f)
            (hlen,) = struct.unpack("<Q", data[:8])
            for name, ent in json.loads(data[8:8 + hlen]).items():
                if name != "__metadata__":
                    a, b = ent["data_offsets"]
                    want[name] = data[8 + hlen + a:8 + hlen + b]
        assert got.keys() == want.keys()
        for k, t in got.items():
            assert t.device.type == "cpu" and t.contiguous().view(torch.uint8).numpy().tobytes() == want[k]
        assert not list((tmp_path / "hf").rglob("*.safetensors")) if (tmp_path / "hf").exists() else True
    finally:
        hub.stop()
