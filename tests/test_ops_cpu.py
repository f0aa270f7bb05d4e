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


def test_host_index_runs_matches_chunk_index_and_reports_errors():
    """_core.index_runs (the engine's host header walk) produces the device kernel's CHUNK_DTYPE
    records for every term, zero records in gaps, and the kernel's error words."""
    import random

    rng = random.Random(4)
    data = rng.randbytes(600_000) + bytes(200_000) + b"xorb index " * 30_000
    ends = C.chunk_ends(data)
    b = C.XorbBuilder("auto")
    prev = 0
    for e in ends:
        b.add_chunk(data[prev:e])
        prev = e
    body = b.serialize(False)
    idx = C.index_chunks(body)
    n = len(idx)
    bounds = b.chunk_boundaries()
    cut = n // 2
    span = np.frombuffer(body + bytes(64), dtype=np.uint8).copy()
    terms = np.zeros(2, dtype=ops.TERM_DTYPE)
    ulen0 = sum(e[3] for e in idx[:cut])
    terms[0] = (0, bounds[cut - 1], 1000, 0, cut, ulen0)
    terms[1] = (bounds[cut - 1], len(body) - bounds[cut - 1], 1000 + ulen0, cut + 3, n - cut,
                len(data) - ulen0)  # 3-record gap before the second term
    out = np.zeros(n + 3, dtype=ops.CHUNK_DTYPE)
    err = C.index_runs(span.ctypes.data, len(body), terms.ctypes.data, 2, out.ctypes.data, len(out))
    assert err == 0
    for i, (hoff, clen, scheme, ulen, uoff) in enumerate(idx):
        r = out[i if i < cut else i + 3]
        assert (int(r["src"]), int(r["clen"]), int(r["scheme"]), int(r["ulen"])) == (hoff + 8, clen, scheme, ulen)
        assert int(r["dst"]) == 1000 + uoff and int(r["term"]) == (0 if i < cut else 1)
    assert not out[cut:cut + 3].view(np.uint8).any()
    # a corrupted header version byte: error code 1 (bad header) for that term, its records zeroed
    bad = span.copy()
    bad[bounds[cut + 1]] = 9
    err = C.index_runs(bad.ctypes.data, len(body), terms.ctypes.data, 2, out.ctypes.data, len(out))
    assert err >> 32 == 1 and err & 0xFFFFFFFF == 1
    assert not out[cut + 3:].view(np.uint8).any() and out[:cut]["clen"].all()
    # a term claiming one chunk more than its bytes hold: count/size mismatch (3)
    t2 = terms.copy()
    t2[0]["n_chunks"] = cut + 1
    t2[0]["ulen"] = 0
    err = C.index_runs(span.ctypes.data, len(body), t2.ctypes.data, 1, out.ctypes.data, len(out))
    assert err >> 32 in (2, 3) and err & 0xFFFFFFFF == 0
