"""Pull a model straight into HBM: every safetensors file is loaded onto the GPU and verified there
against its Xet file hash (GPU CDC + BLAKE3 + Merkle), then exposed as torch tensors.

Single GPU:   python examples/device_tensors.py meta-llama/Llama-3.1-8B
All 8 GPUs:   torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/device_tensors.py <repo> all
              (each file is read from disk by one rank and replicated over xGMI with RCCL)
"""
import sys

import torch

import zest_amd as zest
from zest_amd.parallel import init_from_env

repo = sys.argv[1] if len(sys.argv) > 1 else "openai-community/gpt2"
mode = sys.argv[2] if len(sys.argv) > 2 else "single"
if mode == "all":
    rank, world, local, dev = init_from_env()
    weights = zest.pull(repo, device="all")
else:
    rank, dev = 0, torch.device("cuda:0")
    weights = zest.pull(repo, device=dev)
total = sum(t.numel() * t.element_size() for t in weights.values())
print(f"rank {rank}: {len(weights)} tensors, {total / 1e9:.2f} GB resident on {dev}")
