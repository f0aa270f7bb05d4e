"""Property/fuzz tests (hypothesis) for every decoder that parses untrusted bytes: bencode, BT wire
frames, BEP XET messages, extension handshakes, tracker responses, KRPC compact nodes, LZ4 frames,
xorb chunk runs, reconstruction JSON.  Decoders must either return or raise ZestError — never
crash, hang or read out of bounds (the host build used here is the same code the CLI runs; run
`python tools/build.py --asan` + these tests for sanitizer coverage)."""
from __future__ import annotations

import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from zest_amd import _core  # noqa: E402
from zest_amd._core import ZestError, bencode, bep_xet, bt, dht, tracker  # noqa: E402

FUZZ = settings(max_examples=400, deadline=None)

bvalues = st.recursive(
    st.integers(min_value=-(2**63), max_value=2**63 - 1) | st.binary(max_size=40),
    lambda kids: st.lists(kids, max_size=5) | st.dictionaries(st.binary(max_size=8), kids, max_size=5),
    max_leaves=20,
)


def _safe(fn, *a):
    try:
        fn(*a)
    except ZestError:
        pass


@FUZZ
@given(bvalues)
def test_bencode_roundtrip_property(v):
    enc = bencode.encode(v)
    assert bencode.decode(enc) == v
    assert bencode.encode(bencode.decode(enc)) == enc


@FUZZ
@given(st.binary(max_size=300))
def test_bencode_decoder_total(data):
    _safe(bencode.decode, data)
    _safe(bencode.decode_prefix, data)


@FUZZ
@given(st.binary(max_size=200))
def test_wire_decoders_total(data):
    _safe(bt.parse_message, data)
    _safe(bt.parse_extended, data)
    _safe(bep_xet.decode, data)
    bep_xet.parse_ext_handshake(data)  # documented never to throw
    if len(data) >= 68:
        _safe(bt.parse_handshake, data[:68])


@FUZZ
@given(st.binary(max_size=300))
def test_tracker_and_dht_parsers_total(data):
    _safe(tracker.parse_announce, data)
    _safe(tracker.parse_compact_peers, data)
    _safe(dht.parse_compact_nodes, data)


@FUZZ
@given(st.binary(max_size=2000))
def test_lz4_and_xorb_decoders_total(data):
    _safe(_core.lz4_decompress_frame, data) if hasattr(_core, "lz4_decompress_frame") else None
    _safe(_core.index_chunks, data)
    _safe(_core.parse_footer, data)
    _safe(_core.extract_chunk_range, data, 0, 1, True)


@FUZZ
@given(st.binary(min_size=1, max_size=5000), st.sampled_from(["none", "lz4", "bg4", "auto"]))
def test_xorb_builder_reader_roundtrip(payload, policy):
    b = _core.XorbBuilder(policy)
    b.add_chunk(payload)
    b.add_chunk(payload[::-1])
    blob = b.serialize(True)
    out = _core.extract_chunk_range(blob, 0, 2, True)
    data = out[0] if isinstance(out, tuple) else out
    assert bytes(data) == payload + payload[::-1]


@FUZZ
@given(st.text(max_size=300))
def test_reconstruction_json_parser_total(text):
    _safe(_core.parse_reconstruction, text)


@FUZZ
@given(st.binary(min_size=32, max_size=32), st.integers(min_value=1, max_value=65535))
def test_bep_xet_request_roundtrip(h, rid):
    msg = bep_xet.chunk_request(3, rid, h, 1, 9)
    d = bep_xet.decode(msg[6:])
    assert d["hash"] == h and d["request_id"] == rid
