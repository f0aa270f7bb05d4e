"""The offline fake Hub itself: metadata-only publishing (add_world(payload=False)) serves the same
listing and reconstructions as a full publish, and refuses xorb payloads."""
from __future__ import annotations

import json
import urllib.error
import urllib.request

from zest_amd import models
from zest_amd.synthetic import SyntheticWorld
from zest_amd.testing import FakeHub


def _get(hub, path):
    tok = f"xet-{hub.token}" if path.startswith("/v1/") else hub.token  # CAS uses the xet read token
    req = urllib.request.Request(hub.url + path, headers={"Authorization": f"Bearer {tok}"})
    with urllib.request.urlopen(req, timeout=10) as r:
        return json.loads(r.read())


def test_metadata_only_world_matches_full_publish():
    spec = models.get("llama-tiny")
    w1 = SyntheticWorld(spec, seed=2, max_xorb_bytes=1 << 20)
    w1.build_on_host()
    w2 = SyntheticWorld(spec, seed=2, max_xorb_bytes=1 << 20)
    w2.build_on_host()
    full, meta = FakeHub(), FakeHub()
    full.start()
    meta.start()
    try:
        c1 = full.add_world(w1, exact=True)
        c2 = meta.add_world(w2, exact=True, payload=False)
        assert c1 == c2
        t1 = _get(full, f"/api/models/{spec.repo_id}/tree/main?recursive=true")
        t2 = _get(meta, f"/api/models/{spec.repo_id}/tree/main?recursive=true")
        assert [(e["path"], e["size"], e.get("xetHash")) for e in t1] == \
               [(e["path"], e["size"], e.get("xetHash")) for e in t2]
        for e in t1:
            if not e.get("xetHash"):
                continue
            r1 = _get(full, f"/v1/reconstructions/{e['xetHash']}")
            r2 = _get(meta, f"/v1/reconstructions/{e['xetHash']}")
            assert r1["terms"] == r2["terms"]
            url = next(iter(r2["fetch_info"].values()))[0]["url"]
            try:
                urllib.request.urlopen(url, timeout=10)
                raise AssertionError("metadata-only xorb served")
            except urllib.error.HTTPError as err:
                assert err.code == 404
        assert meta.counters.get("xorb_missing", 0) >= 1
    finally:
        full.stop()
        meta.stop()
