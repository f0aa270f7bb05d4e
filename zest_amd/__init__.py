"""zest_amd — MI355X-native P2P model distribution (zest capabilities, rebuilt for AMD CDNA4).

Layers (see docs/ARCHITECTURE.md):
  zest_amd._core    C++17 host core: BLAKE3/Xet hashing, LZ4/BG4, CDC, xorbs, BT/DHT/HTTP stack
  zest_amd._hip     HIP/CDNA4 kernels for gfx950: xorb ingest (decode+verify), BLAKE3, Merkle, CDC
  zest_amd.ops      torch-facing wrappers of the HIP kernels
  zest_amd.parallel RCCL (torch.distributed "nccl") intra-node swarm: GPUs as BitTorrent peers
  zest_amd.models   synthetic model specs (gpt2, Llama-3.1-8B/70B, Qwen2-7B, Mixtral-8x7B)
  zest_amd.utils    config, safetensors views, tracing, fault injection
"""
from __future__ import annotations

__version__ = "0.4.2"
