"""CPU paths of zest_amd.ops (the host oracle used by gloo multi-process tests)."""
import random

import numpy as np
import torch

from zest_amd import _core as C
from zest_amd import ops


def test_ingest_cpu_path_and_merkle():
    rng = random.Random(2)
    data = rng.randbytes(600_000) + b"abc" * 50_000
    ends = C.chunk_ends(data)
    b = C.XorbBuilder("auto")
    prev = 0
    for e in ends:
        b.add_chunk(data[prev:e])
        prev = e
    body = b.serialize(False)
    src = torch.frombuffer(bytearray(body), dtype=torch.uint8)
    terms = np.zeros(1, dtype=ops.TERM_DTYPE)
    terms[0] = (0, len(body), 5, 0, len(ends), len(data))
    dst = torch.zeros(len(data) + 10, dtype=torch.uint8)
    hashes = torch.zeros((len(ends), 32), dtype=torch.uint8)
    ops.ingest_terms(src, dst, terms, hashes)
    assert dst.numpy().tobytes()[5:5 + len(data)] == data
    assert hashes.numpy().tobytes() == b"".join(b.chunk_hashes())
    sizes = torch.tensor(np.diff([0] + ends), dtype=torch.int64)
    roots = ops.merkle_roots(hashes, sizes, [(0, len(ends))])
    assert roots[0].numpy().tobytes() == C.xet_file_hash(data)


def test_select_boundaries_equals_chunker():
    rng = random.Random(3)
    data = rng.randbytes(2_000_000) + bytes(400_000)
    cand = np.array([i + 1 for i in range(len(data)) if False], dtype=np.uint64)  # placeholder
    # candidates from the host gear hash
    import itertools
    table = ops._gear_table()
    h = 0
    cands = []
    for i, x in enumerate(data):
        h = ((h << 1) + table[x]) & 0xFFFFFFFFFFFFFFFF
        if h & ops.XET_MASK == 0:
            cands.append(i + 1)
    ends = ops.select_chunks(np.array(cands, dtype=np.uint64), len(data))
    assert list(map(int, ends)) == C.chunk_ends(data)
