"""Unit tests of the native wire/protocol codecs, through the pybind11 bindings.

Coverage mirrors the reference's in-file Zig tests (src/bencode.zig:240-368, bt_wire.zig:160-274,
bep_xet.zig:240-362, peer_id.zig:35-63, bt_tracker.zig:184-260, dht.zig:475-671,
main.zig:781-805, config.zig:160-183, bench.zig:291-311) with independently written vectors, plus
the cases where this implementation deliberately differs (strict unknown-id handling, bounded
nesting, canonical key order).
"""
from __future__ import annotations

import hashlib
import json
import struct

import pytest

from zest_amd import _core
from zest_amd._core import ZestError, bencode, bep_xet, bt, dht, tracker


def _err(fn, *a):
    with pytest.raises(ZestError) as ei:
        fn(*a)
    return ei.value.code


# ------------------------------------------------------------------------------------ bencode
@pytest.mark.parametrize("raw,val", [(b"i42e", 42), (b"i-17e", -17), (b"i0e", 0), (b"4:spam", b"spam"), (b"0:", b""),
                                     (b"l4:spami42ee", [b"spam", 42]), (b"le", []), (b"de", {}),
                                     (b"d3:bar4:spam3:fooi42ee", {b"bar": b"spam", b"foo": 42}),
                                     (b"i9223372036854775807e", 2**63 - 1)])
def test_bencode_roundtrip(raw, val):
    assert bencode.decode(raw) == val
    assert bencode.encode(val) == raw
    assert bencode.roundtrip(raw) == raw


@pytest.mark.parametrize("raw,code", [(b"i03e", "LeadingZero"), (b"i-0e", "NegativeZero"),
                                      (b"d3:foo1:a3:bar1:be", "UnsortedDictKeys"), (b"d1:a1:x1:a1:ye", "UnsortedDictKeys"),
                                      (b"i12", "UnexpectedEnd"), (b"5:abc", "UnexpectedEnd"), (b"l", "UnexpectedEnd"),
                                      (b"x", "InvalidFormat"), (b"ie", "InvalidInteger"), (b"i1-2e", "InvalidInteger")])
def test_bencode_rejects(raw, code):
    assert _err(bencode.decode, raw) == code


def test_bencode_nested_and_depth_limit():
    doc = b"d4:infod6:lengthi1024e4:name8:file.binee"
    assert bencode.decode(doc) == {b"info": {b"length": 1024, b"name": b"file.bin"}}
    deep = b"l" * 200 + b"e" * 200
    with pytest.raises(ZestError):
        bencode.decode(deep)
    ok = b"l" * 32 + b"e" * 32
    assert bencode.encode(bencode.decode(ok)) == ok


def test_bencode_encoder_sorts_keys_and_prefix_decode():
    assert bencode.encode({"v": "zest", "m": {"ut_xet": 1}, "p": 6881}) == b"d1:md6:ut_xeti1ee1:pi6881e1:v4:zeste"
    val, used = bencode.decode_prefix(b"i5etrailing")
    assert val == 5 and used == 3


# -------------------------------------------------------------------------------- peer id / SHA1
def test_peer_id_and_info_hash():
    a, b = _core.generate_peer_id(), _core.generate_peer_id()
    assert len(a) == 20 and a[:8] == _core.CLIENT_PREFIX.encode() and a != b
    h = bytes(range(32))
    ih = _core.info_hash(h)
    assert len(ih) == 20 and ih == _core.info_hash(h)
    assert ih == hashlib.sha1(b"zest-xet-v1:" + h).digest()
    assert _core.info_hash(bytes(32)) != _core.info_hash(b"\x01" + bytes(31))
    for n in (0, 1, 55, 56, 63, 64, 65, 1000):
        msg = bytes((i * 7) & 0xFF for i in range(n))
        assert _core.sha1(msg) == hashlib.sha1(msg).digest()


# ------------------------------------------------------------------------------------ BT wire
def test_handshake_roundtrip_and_bep10_bit():
    ih, pid = bytes(range(20)), _core.generate_peer_id()
    hs = bt.handshake(ih, pid)
    assert len(hs) == bt.HANDSHAKE_LEN == 68
    assert hs[0] == 19 and hs[1:20] == b"BitTorrent protocol"
    assert hs[20 + 5] & 0x10
    d = bt.parse_handshake(hs)
    assert d["info_hash"] == ih and d["peer_id"] == pid and d["bep10"]
    bad = b"\x13" + b"BitTorrent protocoX" + hs[20:]
    assert _err(bt.parse_handshake, bad) == "InvalidProtocolString"


def test_message_framing():
    m = bt.message(6, b"\x00" * 12)
    assert m[:4] == struct.pack(">I", 13) and m[4] == 6
    d = bt.parse_message(m + b"extra")
    assert d["consumed"] == len(m) and d["id"] == 6 and d["payload"] == b"\x00" * 12
    assert bt.parse_message(m[:7]) is None  # incomplete frame
    ka = bt.keepalive()
    assert ka == b"\x00\x00\x00\x00" and bt.parse_message(ka)["keepalive"]
    empty = bt.message(2, b"")
    assert empty == b"\x00\x00\x00\x01\x02" and bt.parse_message(empty)["payload"] == b""
    ext = bt.extended(3, b"hello")
    assert ext[4] == 20 and bt.parse_extended(bt.parse_message(ext)["payload"]) == (3, b"hello")
    assert bt.frame_length(struct.pack(">I", 300)) == 304


def test_message_limits_and_unknown_ids():
    huge = struct.pack(">I", bt.MAX_MESSAGE + 1) + b"\x07"
    assert _err(bt.parse_message, huge) == "InvalidMessageSize"
    # unknown id: an error, never undefined behaviour (reference casts to an exhaustive enum)
    assert _err(bt.parse_message, b"\x00\x00\x00\x01\x63") == "InvalidMessageId"
    assert not bt.known_msg_id(99) and bt.known_msg_id(20)


# ------------------------------------------------------------------------------------ BEP XET
def test_bep_xet_messages():
    h = bytes(range(32))
    req = bep_xet.chunk_request(5, 77, h, 3, 9)
    assert len(req) == 6 + 45 and req[4] == 20 and req[5] == 5
    d = bep_xet.decode(req[6:])
    assert d == {"type": bep_xet.CHUNK_REQUEST, "request_id": 77, "hash": h, "range_start": 3, "range_end": 9}
    resp = bep_xet.chunk_response(5, 77, 3, b"payload")
    assert len(resp) == 6 + 13 + 7
    d = bep_xet.decode(resp[6:])
    assert d["type"] == bep_xet.CHUNK_RESPONSE and d["chunk_offset"] == 3 and d["data"] == b"payload"
    nf = bep_xet.chunk_not_found(5, 78, h)
    assert len(nf) == 6 + 37 and bep_xet.decode(nf[6:])["hash"] == h
    er = bep_xet.chunk_error(5, 79, 2, "boom")
    d = bep_xet.decode(er[6:])
    assert d["error_code"] == 2 and d["message"] == b"boom"
    assert _err(bep_xet.decode, b"\x09" + bytes(12)) == "UnknownXetType"
    assert _err(bep_xet.decode, req[6:20]) == "UnexpectedEnd"


def test_ext_handshake():
    raw = bep_xet.make_ext_handshake(6881)
    assert bencode.decode(raw) == {b"m": {b"ut_xet": 1}, b"p": 6881, b"v": b"zest/0.4"}
    assert bep_xet.parse_ext_handshake(raw) == {"ut_xet": 1, "port": 6881, "client": "zest/0.4"}
    other = bencode.encode({"m": {"ut_metadata": 2, "ut_xet": 7}, "p": 51413, "v": "other/1.0"})
    assert bep_xet.parse_ext_handshake(other)["ut_xet"] == 7
    assert bep_xet.parse_ext_handshake(b"garbage")["ut_xet"] == -1


# ------------------------------------------------------------------------------------ tracker
def test_percent_encoding():
    assert _core.percent_encode(bytes([0x00, 0x12, 0xAB, 0xFF])) == "%00%12%AB%FF"
    assert _core.percent_encode(b"AZaz09-._~") == "AZaz09-._~"
    assert _core.percent_decode("%41b%7e") == b"Ab~"


def test_tracker_announce_url_and_parse():
    ih, pid = bytes([0xAA] * 20), b"-ZE0402-" + b"0" * 12
    url = tracker.announce_url("http://t.example/announce", ih, pid, 6881, "started")
    assert url.startswith("http://t.example/announce?info_hash=" + "%AA" * 20)
    for part in ("port=6881", "compact=1", "event=started", "peer_id=-ZE0402-"):
        assert part in url
    compact = bytes([10, 0, 0, 5, 0x1A, 0xE1, 192, 168, 1, 2, 0x1F, 0x90])
    r = tracker.parse_announce(bencode.encode({"interval": 900, "peers": compact}))
    assert r == {"interval": 900, "peers": ["10.0.0.5:6881", "192.168.1.2:8080"]}
    # dict-model peers too
    r = tracker.parse_announce(bencode.encode({"peers": [{"ip": "1.2.3.4", "port": 5}]}))
    assert r["peers"] == ["1.2.3.4:5"] and r["interval"] == 1800
    assert _err(tracker.parse_announce, bencode.encode({"failure reason": "nope"})) == "TrackerError"
    assert tracker.parse_compact_peers(compact) == ["10.0.0.5:6881", "192.168.1.2:8080"]
    assert tracker.encode_compact_peer("10.0.0.5:6881") == compact[:6]


# ------------------------------------------------------------------------------------ DHT
def test_dht_metric_and_buckets():
    a, b = bytes(20), bytes([0x80]) + bytes(19)
    assert dht.xor_distance(a, b) == b
    assert dht.bucket_index(a, b) == 0  # highest bit differs (reference dht.zig:497-509 convention)
    assert dht.bucket_index(a, bytes(19) + b"\x01") == 159
    assert dht.bucket_index(a, a) == -1


def test_routing_table_insert_full_closest():
    own = bytes(20)
    t = dht.RoutingTable(own)
    ids = [bytes([0x80 | i]) + bytes(19) for i in range(10)]  # all in bucket 0
    ins = [t.insert(i, f"127.0.0.1:{1000 + k}") for k, i in enumerate(ids)]
    assert ins[:8] == [True] * 8 and ins[8:] == [False, False]  # full bucket keeps old nodes
    assert len(t) == 8
    t.remove(ids[0])
    assert len(t) == 7
    near = bytes(19) + b"\x05"
    t.insert(near, "127.0.0.1:2000")
    closest = t.closest(bytes(20), 3)
    assert closest[0] == (near, "127.0.0.1:2000") and len(closest) == 3


def test_krpc_encoding_and_compact_nodes():
    own, ih = bytes(range(20)), bytes(range(20, 40))
    ping = bencode.decode(dht.build_ping(b"aa", own))
    assert ping == {b"a": {b"id": own}, b"q": b"ping", b"t": b"aa", b"y": b"q"}
    gp = bencode.decode(dht.build_get_peers(b"bb", own, ih))
    assert gp[b"q"] == b"get_peers" and gp[b"a"][b"info_hash"] == ih
    ap = bencode.decode(dht.build_announce_peer(b"cc", own, ih, 6881, b"tok"))
    assert ap[b"a"][b"port"] == 6881 and ap[b"a"][b"token"] == b"tok"
    node = dht.encode_compact_node(own, "10.1.2.3:6881")
    assert len(node) == 26
    assert dht.parse_compact_nodes(node * 2) == [(own, "10.1.2.3:6881")] * 2
    assert dht.parse_compact_nodes(node[:25]) == []


def test_dht_nodes_find_each_other():
    a, b, c = dht.Node(0), dht.Node(0), dht.Node(0)
    try:
        assert b.bootstrap([f"127.0.0.1:{a.port}"]) >= 1
        assert c.bootstrap([f"127.0.0.1:{a.port}"]) >= 1
        ih = bytes([7] * 20)
        assert b.announce_peer(ih, 4242) >= 1
        peers = c.get_peers(ih)
        assert "127.0.0.1:4242" in peers
        assert a.ping(f"127.0.0.1:{b.port}")
        assert c.stats()["lookups"] >= 1
    finally:
        for n in (a, b, c):
            n.stop()


# ------------------------------------------------------------------------------------ misc
def test_extract_json_sha():
    sha = "607a30d783dfa663caf39e06633721c8d4cfcd7e"
    assert _core.extract_json_sha('{"_id":"x","sha":"%s","siblings":[]}' % sha) == sha
    assert _core.extract_json_sha('{"id":"x"}') is None
    assert _core.extract_json_sha('{"sha":"zzzz30d783dfa663caf39e06633721c8d4cfcd7e"}') is None


def test_config_env(monkeypatch, tmp_path):
    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.delenv("HF_HOME", raising=False)
    monkeypatch.delenv("HF_HUB_CACHE", raising=False)
    monkeypatch.delenv("ZEST_CACHE_DIR", raising=False)
    monkeypatch.setenv("ZEST_HTTP_PORT", "12345")
    monkeypatch.setenv("HF_TOKEN", "hf_abc")
    c = json.loads(_core.config_json())
    assert c["hf_cache_dir"] == f"{tmp_path}/.cache/huggingface/hub"
    assert c["xorb_cache_dir"] == f"{tmp_path}/.cache/zest/xorbs"
    assert c["http_port"] == 12345 and c["listen_port"] == 6881 and c["max_peers"] == 50
    assert c["has_token"] is True
    monkeypatch.setenv("HF_HOME", str(tmp_path / "hfh"))
    assert json.loads(_core.config_json())["hf_cache_dir"] == f"{tmp_path}/hfh/hub"
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "hub2"))
    assert json.loads(_core.config_json())["hf_cache_dir"] == f"{tmp_path}/hub2"
    assert _core.repo_folder_name("meta-llama/Llama-3.1-8B") == "models--meta-llama--Llama-3.1-8B"
    assert _core.repo_folder_name("org/ds", "dataset") == "datasets--org--ds"


def test_bench_rows():
    rows = _core.bench_synthetic(False)
    assert [r["name"] for r in rows] == ["bencode_encode", "bencode_decode", "blake3_64kb", "sha1_info_hash",
                                         "bt_wire_frame"]
    for r in rows:
        assert r["median_ns"] > 0 and r["throughput_mbps"] > 0


def test_reconstruction_json_roundtrip():
    rec = {"offset_into_first_range": 0,
           "terms": [{"hash": "ab" * 32, "unpacked_length": 100, "range": {"start": 0, "end": 2}}],
           "fetch_info": {"ab" * 32: [{"range": {"start": 0, "end": 2}, "url": "http://x/y",
                                       "url_range": {"start": 0, "end": 99}}]}}
    back = json.loads(_core.parse_reconstruction(json.dumps(rec)))
    assert back["terms"][0]["unpacked_length"] == 100
    assert back["fetch_info"]["ab" * 32][0]["url_range"] == {"start": 0, "end": 99}


def test_seeder_caps_inbound_connections(monkeypatch, tmp_path):
    """ZEST_MAX_INBOUND bounds the seeding server's connection threads: a peer past the cap is
    closed at accept (counted in stats()["rejected"]); once a served peer leaves, a new one is
    served again."""
    import socket
    import time

    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.setenv("ZEST_CACHE_DIR", str(tmp_path / "zc"))
    monkeypatch.setenv("ZEST_MAX_INBOUND", "2")
    seeder = _core.Seeder(port=0)

    def wait_for(pred, what):
        for _ in range(200):
            if pred():
                return
            time.sleep(0.025)
        raise AssertionError(f"timed out waiting for {what}: {seeder.stats()}")

    def closed_by_server(sock):
        sock.settimeout(5)
        try:
            return sock.recv(1) == b""
        except ConnectionResetError:
            return True

    try:
        held = [socket.create_connection(("127.0.0.1", seeder.port)) for _ in range(2)]
        wait_for(lambda: seeder.stats()["active_peers"] == 2, "two served peers")
        extra = socket.create_connection(("127.0.0.1", seeder.port))
        assert closed_by_server(extra)
        extra.close()
        wait_for(lambda: seeder.stats()["rejected"] == 1, "one rejected peer")
        held.pop().close()
        wait_for(lambda: seeder.stats()["active_peers"] == 1, "the closed peer's thread to end")
        again = socket.create_connection(("127.0.0.1", seeder.port))
        wait_for(lambda: seeder.stats()["active_peers"] == 2, "the new peer to be served")
        assert seeder.stats()["rejected"] == 1
        again.close()
        for s in held:
            s.close()
    finally:
        seeder.stop()
