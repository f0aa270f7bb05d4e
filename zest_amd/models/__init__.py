"""Synthetic model families for benchmarks and offline tests (random-init weights, real shapes).

The reference distributes HuggingFace checkpoints; its benchmark configs (BASELINE.json) name
gpt2, Llama-3.1-8B, Llama-3.1-70B, Qwen2-7B and Mixtral-8x7B.  With no network, we materialize
those repositories synthetically: the exact tensor names/shapes/dtypes of each architecture,
sharded into `model-0000k-of-0000n.safetensors` files the way HF's `save_pretrained` does
(max_shard_size 5 GB), plus config.json / generation_config.json so `from_pretrained` accepts the
snapshot.  Weight bytes come from a deterministic generator (zest_amd.ops.fill_synthetic on the
GPU, or numpy on the CPU): mode "random" = uniform random bytes (BASELINE's "random-byte
weights"), mode "bf16" = bf16 ~ N(0, 0.02) (compressible with BG4-LZ4 like real checkpoints).
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field

DTYPE_BYTES = {"BF16": 2, "F16": 2, "F32": 4, "I64": 8}


@dataclass
class TensorSpec:
    name: str
    dtype: str
    shape: tuple

    @property
    def nbytes(self) -> int:
        n = DTYPE_BYTES[self.dtype]
        for s in self.shape:
            n *= s
        return n


@dataclass
class ShardFile:
    path: str
    tensors: list  # TensorSpec in file order
    header: bytes = b""  # 8-byte length + JSON (padded to 8)
    offsets: dict = field(default_factory=dict)  # name -> (begin, end) relative to data start

    @property
    def data_bytes(self) -> int:
        return sum(t.nbytes for t in self.tensors)

    @property
    def size(self) -> int:
        return len(self.header) + self.data_bytes


@dataclass
class ModelSpec:
    repo_id: str
    arch: str
    config: dict
    tensors: list
    dtype: str = "BF16"
    max_shard_bytes: int = 5 * 10**9
    extra_files: dict = field(default_factory=dict)  # small regular files: path -> bytes

    @property
    def n_params(self) -> int:
        total = 0
        for t in self.tensors:
            n = 1
            for s in t.shape:
                n *= s
            total += n
        return total

    @property
    def nbytes(self) -> int:
        return sum(t.nbytes for t in self.tensors)

    def shards(self) -> list[ShardFile]:
        """HF save_pretrained-style sharding (greedy by tensor order, <= max_shard_bytes)."""
        groups, cur, cur_b = [], [], 0
        for t in self.tensors:
            if cur and cur_b + t.nbytes > self.max_shard_bytes:
                groups.append(cur)
                cur, cur_b = [], 0
            cur.append(t)
            cur_b += t.nbytes
        if cur:
            groups.append(cur)
        n = len(groups)
        out = []
        for i, g in enumerate(groups):
            name = "model.safetensors" if n == 1 else f"model-{i + 1:05d}-of-{n:05d}.safetensors"
            sf = ShardFile(name, g)
            sf.header, sf.offsets = safetensors_header(g)
            out.append(sf)
        return out

    def index_json(self, shards: list[ShardFile]) -> bytes | None:
        if len(shards) == 1:
            return None
        wm = {t.name: s.path for s in shards for t in s.tensors}
        return json.dumps({"metadata": {"total_size": self.nbytes}, "weight_map": wm}, indent=2).encode()

    def small_files(self, shards: list[ShardFile]) -> dict[str, bytes]:
        files = {"config.json": json.dumps(self.config, indent=2).encode(),
                 "generation_config.json": json.dumps({"_from_model_config": True}).encode()}
        idx = self.index_json(shards)
        if idx is not None:
            files["model.safetensors.index.json"] = idx
        files.update(self.extra_files)
        return files


def safetensors_header(tensors: list[TensorSpec]) -> tuple[bytes, dict]:
    meta = {"__metadata__": {"format": "pt"}}
    offsets = {}
    pos = 0
    for t in tensors:
        meta[t.name] = {"dtype": t.dtype, "shape": list(t.shape), "data_offsets": [pos, pos + t.nbytes]}
        offsets[t.name] = (pos, pos + t.nbytes)
        pos += t.nbytes
    js = json.dumps(meta, separators=(",", ":")).encode()
    js += b" " * ((8 - len(js) % 8) % 8)  # 8-byte align the data section
    return struct.pack("<Q", len(js)) + js, offsets


# ------------------------------------------------------------------------------------------------
# Architectures
# ------------------------------------------------------------------------------------------------
def _llama_like(repo_id, *, hidden, inter, layers, heads, kv_heads, vocab, tie=False, bias=False,
                arch="LlamaForCausalLM", model_type="llama", rope_theta=500000.0, max_pos=131072,
                dtype="BF16", extra_cfg=None) -> ModelSpec:
    hd = hidden // heads
    ts = [TensorSpec("model.embed_tokens.weight", dtype, (vocab, hidden))]
    for i in range(layers):
        p = f"model.layers.{i}."
        ts += [TensorSpec(p + "input_layernorm.weight", dtype, (hidden,)),
               TensorSpec(p + "mlp.down_proj.weight", dtype, (hidden, inter)),
               TensorSpec(p + "mlp.gate_proj.weight", dtype, (inter, hidden)),
               TensorSpec(p + "mlp.up_proj.weight", dtype, (inter, hidden)),
               TensorSpec(p + "post_attention_layernorm.weight", dtype, (hidden,)),
               TensorSpec(p + "self_attn.k_proj.weight", dtype, (kv_heads * hd, hidden)),
               TensorSpec(p + "self_attn.o_proj.weight", dtype, (hidden, heads * hd)),
               TensorSpec(p + "self_attn.q_proj.weight", dtype, (heads * hd, hidden)),
               TensorSpec(p + "self_attn.v_proj.weight", dtype, (kv_heads * hd, hidden))]
        if bias:
            ts += [TensorSpec(p + "self_attn.k_proj.bias", dtype, (kv_heads * hd,)),
                   TensorSpec(p + "self_attn.q_proj.bias", dtype, (heads * hd,)),
                   TensorSpec(p + "self_attn.v_proj.bias", dtype, (kv_heads * hd,))]
    ts.append(TensorSpec("model.norm.weight", dtype, (hidden,)))
    if not tie:
        ts.append(TensorSpec("lm_head.weight", dtype, (vocab, hidden)))
    cfg = {"architectures": [arch], "model_type": model_type, "hidden_size": hidden,
           "intermediate_size": inter, "num_hidden_layers": layers, "num_attention_heads": heads,
           "num_key_value_heads": kv_heads, "vocab_size": vocab, "rms_norm_eps": 1e-5,
           "rope_theta": rope_theta, "max_position_embeddings": max_pos, "tie_word_embeddings": tie,
           "torch_dtype": "bfloat16" if dtype == "BF16" else "float32", "hidden_act": "silu"}
    if extra_cfg:
        cfg.update(extra_cfg)
    return ModelSpec(repo_id, arch, cfg, ts, dtype)


def _mixtral(repo_id, *, hidden=4096, inter=14336, layers=32, heads=32, kv_heads=8, vocab=32000,
             experts=8, dtype="BF16") -> ModelSpec:
    hd = hidden // heads
    ts = [TensorSpec("model.embed_tokens.weight", dtype, (vocab, hidden))]
    for i in range(layers):
        p = f"model.layers.{i}."
        ts.append(TensorSpec(p + "block_sparse_moe.gate.weight", dtype, (experts, hidden)))
        for e in range(experts):
            q = f"{p}block_sparse_moe.experts.{e}."
            ts += [TensorSpec(q + "w1.weight", dtype, (inter, hidden)),
                   TensorSpec(q + "w2.weight", dtype, (hidden, inter)),
                   TensorSpec(q + "w3.weight", dtype, (inter, hidden))]
        ts += [TensorSpec(p + "input_layernorm.weight", dtype, (hidden,)),
               TensorSpec(p + "post_attention_layernorm.weight", dtype, (hidden,)),
               TensorSpec(p + "self_attn.k_proj.weight", dtype, (kv_heads * hd, hidden)),
               TensorSpec(p + "self_attn.o_proj.weight", dtype, (hidden, heads * hd)),
               TensorSpec(p + "self_attn.q_proj.weight", dtype, (heads * hd, hidden)),
               TensorSpec(p + "self_attn.v_proj.weight", dtype, (kv_heads * hd, hidden))]
    ts += [TensorSpec("model.norm.weight", dtype, (hidden,)), TensorSpec("lm_head.weight", dtype, (vocab, hidden))]
    cfg = {"architectures": ["MixtralForCausalLM"], "model_type": "mixtral", "hidden_size": hidden,
           "intermediate_size": inter, "num_hidden_layers": layers, "num_attention_heads": heads,
           "num_key_value_heads": kv_heads, "vocab_size": vocab, "num_local_experts": experts,
           "num_experts_per_tok": 2, "rms_norm_eps": 1e-5, "rope_theta": 1e6,
           "max_position_embeddings": 32768, "torch_dtype": "bfloat16", "tie_word_embeddings": False}
    return ModelSpec(repo_id, "MixtralForCausalLM", cfg, ts, dtype)


def _gpt2(repo_id="openai-community/gpt2", *, layers=12, hidden=768, heads=12, vocab=50257, n_pos=1024,
          dtype="F32") -> ModelSpec:
    ts = [TensorSpec("wte.weight", dtype, (vocab, hidden)), TensorSpec("wpe.weight", dtype, (n_pos, hidden))]
    for i in range(layers):
        p = f"h.{i}."
        ts += [TensorSpec(p + "ln_1.weight", dtype, (hidden,)), TensorSpec(p + "ln_1.bias", dtype, (hidden,)),
               TensorSpec(p + "attn.c_attn.weight", dtype, (hidden, 3 * hidden)),
               TensorSpec(p + "attn.c_attn.bias", dtype, (3 * hidden,)),
               TensorSpec(p + "attn.c_proj.weight", dtype, (hidden, hidden)),
               TensorSpec(p + "attn.c_proj.bias", dtype, (hidden,)),
               TensorSpec(p + "ln_2.weight", dtype, (hidden,)), TensorSpec(p + "ln_2.bias", dtype, (hidden,)),
               TensorSpec(p + "mlp.c_fc.weight", dtype, (hidden, 4 * hidden)),
               TensorSpec(p + "mlp.c_fc.bias", dtype, (4 * hidden,)),
               TensorSpec(p + "mlp.c_proj.weight", dtype, (4 * hidden, hidden)),
               TensorSpec(p + "mlp.c_proj.bias", dtype, (hidden,))]
    ts += [TensorSpec("ln_f.weight", dtype, (hidden,)), TensorSpec("ln_f.bias", dtype, (hidden,))]
    cfg = {"architectures": ["GPT2LMHeadModel"], "model_type": "gpt2", "n_embd": hidden, "n_layer": layers,
           "n_head": heads, "vocab_size": vocab, "n_positions": n_pos, "n_ctx": n_pos,
           "activation_function": "gelu_new", "layer_norm_epsilon": 1e-5, "torch_dtype": "float32"}
    return ModelSpec(repo_id, "GPT2LMHeadModel", cfg, ts, dtype, max_shard_bytes=10**12)


def get(name: str) -> ModelSpec:
    """Model spec by repo id or short alias."""
    key = name.lower()
    if key in ("gpt2", "openai-community/gpt2", "synthetic/gpt2"):
        return _gpt2("openai-community/gpt2" if "synthetic" not in key else "synthetic/gpt2")
    if key in ("gpt2-tiny", "synthetic/gpt2-tiny"):
        return _gpt2("synthetic/gpt2-tiny", layers=2, hidden=64, heads=2, vocab=1000, n_pos=128)
    if key in ("llama-3.1-8b", "meta-llama/llama-3.1-8b", "meta-llama/meta-llama-3.1-8b"):
        return _llama_like("meta-llama/Llama-3.1-8B", hidden=4096, inter=14336, layers=32, heads=32, kv_heads=8,
                           vocab=128256)
    if key in ("llama-3.1-70b", "meta-llama/llama-3.1-70b", "meta-llama/meta-llama-3.1-70b"):
        return _llama_like("meta-llama/Llama-3.1-70B", hidden=8192, inter=28672, layers=80, heads=64, kv_heads=8,
                           vocab=128256)
    if key in ("llama-tiny", "synthetic/llama-tiny"):
        return _llama_like("synthetic/llama-tiny", hidden=256, inter=512, layers=2, heads=4, kv_heads=2, vocab=1024,
                           max_pos=512)
    if key in ("llama-tiny-sharded", "synthetic/llama-tiny-sharded"):  # several files / terms (multi-rank tests)
        spec = _llama_like("synthetic/llama-tiny-sharded", hidden=256, inter=512, layers=4, heads=4, kv_heads=2,
                           vocab=1024, max_pos=512)
        spec.max_shard_bytes = 700_000
        return spec
    if key in ("qwen2-7b", "qwen/qwen2-7b"):
        return _llama_like("Qwen/Qwen2-7B", hidden=3584, inter=18944, layers=28, heads=28, kv_heads=4, vocab=152064,
                           bias=True, arch="Qwen2ForCausalLM", model_type="qwen2", rope_theta=1e6, max_pos=131072)
    if key in ("mixtral-8x7b", "mistralai/mixtral-8x7b-v0.1", "mistralai/mixtral-8x7b"):
        return _mixtral("mistralai/Mixtral-8x7B-v0.1")
    raise KeyError(f"unknown model {name!r}")


ALL = ["gpt2", "llama-3.1-8b", "llama-3.1-70b", "qwen2-7b", "mixtral-8x7b", "gpt2-tiny", "llama-tiny"]
