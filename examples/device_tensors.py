"""Pull a model straight into HBM: every term is fetched (xorb cache -> peers -> CDN) into pinned
staging, copied to the GPU, decoded (LZ4 / BG4) and BLAKE3-hashed there, every file is checked
against its Xet hash (Merkle), and the weights come back as torch tensors -- no disk snapshot unless
save_snapshot=True.

Single GPU:   python examples/device_tensors.py meta-llama/Llama-3.1-8B
All 8 GPUs:   torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/device_tensors.py <repo> all
              (each rank fetches a byte-balanced share of the terms; the shares are replicated over
              xGMI through per-process exchange windows, RCCL as the fallback; every rank verifies
              its whole replica -- zest_amd.parallel.swarm_pull)
One command:  zest pull <repo> --gpus 8 --device all [--save-snapshot]
              (starts the ranks itself: zest_amd/replicate.py)
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
