"""Offline HuggingFace Hub + Xet CAS + BT tracker, for tests and air-gapped demos.

The real services are unreachable from this environment, so the end-to-end tests run the native
client (`zest pull`, `zest_amd.pull`) and the official `hf_xet` client against this server.  It
implements exactly the HTTP surface the clients use:

* Hub:   ``GET /api/{models,datasets}/{repo}/tree/{rev}?recursive=true&expand=true`` (with
  ``xetHash`` per Xet file and RFC 5988 ``Link`` pagination), ``GET /api/models/{repo}/revision/{rev}``
  (``{"sha": ...}``), ``GET /api/models/{repo}/xet-read-token/{rev}`` (``accessToken``,
  ``casUrl``, ``exp``), ``GET /{repo}/resolve/{rev}/{path}``.
* CAS:   ``GET /v1/reconstructions/{file_hash}`` (optionally honouring ``Range: bytes=a-b`` on the
  file), ``/v2/...`` answered 404 so clients fall back to v1, ``GET /xorbs/default/{xorb_hash}``
  with byte ``Range`` support (206).
* Tracker: ``GET /announce`` (BEP 3 / BEP 23 compact peers).

Xet content is produced by our own codec (CDC chunker, BLAKE3 Merkle hashing, xorb serializer with
optional LZ4 / BG4 compression — all pinned byte-for-byte against hf_xet in tests/test_xet_golden.py),
with global chunk dedup like the real CAS, so reconstructions contain multi-xorb files and terms
that reference xorbs shared with other files.

Reference behaviour being emulated: the reference talks to these same endpoints in
src/main.zig:139-256 (hub), src/xet_bridge.zig:60-190 (CAS) and src/bt_tracker.zig:14-80 (tracker).
"""
from __future__ import annotations

import hashlib
import itertools
import json
import threading
import time
import urllib.parse
from dataclasses import dataclass, field
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np

from .. import _core

MAX_XORB_BYTES = 64 << 20
MAX_XORB_CHUNKS = 8192


@dataclass
class _Xorb:
    data: bytes
    hash_hex: str
    boundaries: list[int]          # serialized end offset of each chunk
    ulens: list[int]
    cum: list[int] = field(default_factory=list, repr=False)  # prefix sums of ulens (cum[0] = 0)

    def __post_init__(self):
        self.cum = list(itertools.accumulate(self.ulens, initial=0))


@dataclass
class _File:
    path: str
    data: bytes
    xet_hash: str | None = None
    terms: list[tuple[int, int, int]] = field(default_factory=list)  # (xorb_idx, c0, c1)
    _oid: str | None = None
    _sha256: str | None = None

    def digests(self) -> tuple[str, str]:
        """(git blob oid, sha256), computed once: tree listings of multi-GB repos stay fast."""
        if self._oid is None:
            h = hashlib.sha1(b"blob %d\0" % len(self.data))
            h.update(self.data)
            self._oid = h.hexdigest()
            self._sha256 = hashlib.sha256(self.data).hexdigest()
        return self._oid, self._sha256


class _LazyFile(_File):
    """Xet file published without host bytes (add_world(payload=False)); only its size is known."""

    def __init__(self, path: str, data: bytes, size: int):
        super().__init__(path, data)
        self.size = size


@dataclass
class _Repo:
    repo_id: str
    repo_type: str
    commit: str
    files: dict[str, _File]
    revisions: dict[str, str]


class FakeHub:
    """In-process fake of huggingface.co + Xet CAS + a BT tracker (threaded HTTP server)."""

    def __init__(self, policy: str = "none", token: str = "hf_fake_token", require_auth: bool = False,
                 max_xorb_bytes: int = MAX_XORB_BYTES, page_size: int = 0, host: str = "127.0.0.1"):
        self.policy = policy
        self.token = token
        self.require_auth = require_auth
        self.max_xorb_bytes = max_xorb_bytes
        self.page_size = page_size
        self.host = host
        self.repos: dict[tuple[str, str], _Repo] = {}
        self.xorbs: list[_Xorb] = []
        self.xorb_index: dict[str, int] = {}
        self.file_index: dict[str, _File] = {}
        self._recon_cache: dict = {}
        self._chunk_loc: dict[bytes, tuple[int, int]] = {}
        self._open: list[tuple[bytes, bytes]] = []   # (chunk_hash, chunk) of the open xorb
        self._open_ser = 0
        self.lock = threading.Lock()
        self.counters: dict[str, int] = {}
        self.xorb_bytes_served = 0
        self.fail_xorbs: set[str] = set()      # xorb hex -> 500
        self.corrupt_xorbs: set[str] = set()   # xorb hex -> flipped byte in the body
        self.ignore_range = False
        self.xorb_delay_s = 0.0                # slow CDN: sleep before each xorb response
        self.xorb_delay_stagger = 0            # k > 0: the n-th xorb response waits (1 + n % k) x the delay
        self._xorb_gets = 0
        self._delay_lock = threading.Lock()
        self.tracker_peers: dict[bytes, dict[str, float]] = {}
        # Base of the xorb URLs handed out in fetch_info (None: this server's presigned /xorbs/ URLs).
        # "mem://<name>" points the client's CDN fetches at an in-process memory origin
        # (zest_amd.ops.mem_origin_add; the bench's CDN stand-in for the public swarm_pull path).
        self.xorb_url: str | None = None
        self._srv: ThreadingHTTPServer | None = None
        self._thr: threading.Thread | None = None

    # ------------------------------------------------------------------ content
    def add_repo(self, repo_id: str, files: dict[str, bytes], revision: str = "main", repo_type: str = "model",
                 xet_min_size: int = 1, xet_suffixes: tuple[str, ...] | None = None, commit: str | None = None) -> str:
        """Publish `files` as `repo_id@revision`; returns the commit sha.

        Files of at least `xet_min_size` bytes (or matching `xet_suffixes` when given) are Xet-backed;
        the rest are plain LFS-less files served by /resolve.
        """
        commit = commit or hashlib.sha1(repr((repo_id, revision, sorted((k, hashlib.sha256(v).hexdigest())
                                                                        for k, v in files.items()))).encode()).hexdigest()
        out: dict[str, _File] = {}
        with self.lock:
            for path, data in files.items():
                f = _File(path, bytes(data))
                is_xet = (path.endswith(xet_suffixes) if xet_suffixes else len(data) >= xet_min_size) and len(data) > 0
                if is_xet:
                    self._ingest(f)
                out[path] = f
            self._seal()
            for f in out.values():
                if f.terms is not None and f.xet_hash is not None:
                    self.file_index[f.xet_hash] = f
        for f in out.values():
            f.digests()
        key = (repo_type, repo_id)
        if key in self.repos:
            repo = self.repos[key]
            repo.revisions[revision] = commit
            repo.files = out
            repo.commit = commit
        else:
            self.repos[key] = _Repo(repo_id, repo_type, commit, out, {revision: commit, commit: commit})
        self.repos[key].revisions[commit] = commit
        return commit

    def add_world(self, world, revision: str = "main", exact: bool = False, payload: bool = True) -> str:
        """Publish a zest_amd.synthetic.SyntheticWorld (host-generated bytes).

        exact=True reuses the world's own xorb layout (so xorb hashes match what a device-built
        world / HBM seeder holds); otherwise the files are re-packed by this hub like any upload.
        payload=False (exact only) publishes metadata without generating any Xet bytes on the host:
        listings, reconstructions and hashes are real, xorb GETs answer 404 (counted as
        `xorb_missing`), so every byte has to come from peers — used for multi-GB benches where the
        content lives in an HBM seeder."""
        if not payload:
            return self._add_world_metadata(world, revision)
        files = {f.path: world.file_bytes_host(f) for f in world.files}
        if not exact:
            return self.add_repo(world.spec.repo_id, files, revision=revision,
                                 xet_suffixes=(".safetensors",), commit=world.commit)
        if world.terms is None:
            world.build_on_host()
        if world.chunk_scheme is not None and world.chunk_scheme.any():
            raise ValueError("exact publishing of a compressed world needs payload=False (bytes from an HBM seeder)")
        contents = {f.path: files[f.path] for f in world.xet_files}
        base = len(self.xorbs)
        with self.lock:
            for x in range(world.n_xorbs):
                data = world.xorb_bytes_host(x, contents, policy="none", footer=True)
                a = int(world.xorb_chunk0[x])
                b = int(world.xorb_chunk0[x + 1]) if x + 1 < world.n_xorbs else world.n_chunks
                ser = world.chunk_len[a:b].astype(np.int64) + 8
                hx = world.xorb_hash_hex(x)
                self.xorbs.append(_Xorb(data, hx, np.cumsum(ser).tolist(), world.chunk_len[a:b].tolist()))
                self.xorb_index[hx] = base + x
            out = {}
            for i, f in enumerate(world.files):
                ff = _File(f.path, files[f.path])
                if f.xet:
                    fi = world.xet_files.index(f)
                    T = world.terms[world.terms["file"] == fi]
                    ff.xet_hash = world.file_hash_hex(fi)
                    ff.terms = [(base + int(t["xorb"]), int(t["local0"]), int(t["local0"] + t["c1"] - t["c0"]))
                                for t in T]
                    self.file_index[ff.xet_hash] = ff
                out[f.path] = ff
        for ff in out.values():
            ff.digests()
        key = ("model", world.spec.repo_id)
        self.repos[key] = _Repo(world.spec.repo_id, "model", world.commit, out,
                                {revision: world.commit, world.commit: world.commit})
        return world.commit

    def _add_world_metadata(self, world, revision: str) -> str:
        if world.terms is None:
            raise ValueError("build the world (build_on_device / build_on_host) first")
        base = len(self.xorbs)
        with self.lock:
            # serialized sizes: header + STORED payload (a compressed world's chunks are LZ4/BG4 frames)
            stored = world.chunk_clen if world.chunk_clen is not None else world.chunk_len
            for x in range(world.n_xorbs):
                a = int(world.xorb_chunk0[x])
                b = int(world.xorb_chunk0[x + 1]) if x + 1 < world.n_xorbs else world.n_chunks
                ser = stored[a:b].astype(np.int64) + 8
                hx = world.xorb_hash_hex(x)
                self.xorbs.append(_Xorb(None, hx, np.cumsum(ser).tolist(), world.chunk_len[a:b].tolist()))
                self.xorb_index[hx] = base + x
            out = {}
            for f in world.files:
                if f.xet:
                    fi = world.xet_files.index(f)
                    ff = _LazyFile(f.path, b"", size=f.size)
                    ff.xet_hash = world.file_hash_hex(fi)
                    T = world.terms[world.terms["file"] == fi]
                    ff.terms = [(base + int(t["xorb"]), int(t["local0"]), int(t["local0"] + t["c1"] - t["c0"]))
                                for t in T]
                    # no bytes on the host: stand-in digests derived from the Xet hash
                    ff._oid = hashlib.sha1(ff.xet_hash.encode()).hexdigest()
                    ff._sha256 = hashlib.sha256(ff.xet_hash.encode()).hexdigest()
                    self.file_index[ff.xet_hash] = ff
                else:
                    ff = _File(f.path, f.content)
                    ff.digests()
                out[f.path] = ff
        key = ("model", world.spec.repo_id)
        self.repos[key] = _Repo(world.spec.repo_id, "model", world.commit, out,
                                {revision: world.commit, world.commit: world.commit})
        return world.commit

    def _ingest(self, f: _File) -> None:
        data = f.data
        ends = _core.chunk_ends(data)
        leaves = []
        locs = []
        prev = 0
        for e in ends:
            chunk = data[prev:e]
            h = _core.chunk_hash(chunk)
            leaves.append((h, e - prev))
            loc = self._chunk_loc.get(h)
            if loc is None:
                loc = self._append_chunk(h, chunk)
            locs.append(loc)
            prev = e
        f.xet_hash = _core.xet_hex(_core.file_hash(leaves))
        f.terms = []
        # xorb indices for the open xorb are provisional (-1 - k) until sealed
        f._locs = locs  # type: ignore[attr-defined]
        self._pending = getattr(self, "_pending", [])
        self._pending.append(f)

    def _append_chunk(self, h: bytes, chunk: bytes) -> tuple[int, int]:
        ser = len(chunk) + 8 + 64  # upper bound (compression never expands past header + raw)
        if self._open and (len(self._open) >= MAX_XORB_CHUNKS or self._open_ser + ser > self.max_xorb_bytes):
            self._seal_open()
        self._open.append((h, chunk))
        self._open_ser += ser
        loc = (-1 - len(self.xorbs), len(self._open) - 1)  # provisional: xorb being built
        self._chunk_loc[h] = loc
        return loc

    def _seal_open(self) -> None:
        if not self._open:
            return
        b = _core.XorbBuilder(self.policy)
        for _, c in self._open:
            b.add_chunk(c)
        data = b.serialize(True)
        hx = _core.xet_hex(b.hash())
        idx = len(self.xorbs)
        self.xorbs.append(_Xorb(data, hx, list(b.chunk_boundaries()), list(b.chunk_ulens())))
        self.xorb_index[hx] = idx
        for k, (h, _) in enumerate(self._open):
            self._chunk_loc[h] = (idx, k)
        self._open = []
        self._open_ser = 0

    def _seal(self) -> None:
        self._seal_open()
        for f in getattr(self, "_pending", []):
            terms: list[tuple[int, int, int]] = []
            for (x, c) in f._locs:  # type: ignore[attr-defined]
                if x < 0:
                    x = -1 - x
                if terms and terms[-1][0] == x and terms[-1][2] == c:
                    terms[-1] = (x, terms[-1][1], c + 1)
                else:
                    terms.append((x, c, c + 1))
            f.terms = terms
            del f._locs  # type: ignore[attr-defined]
        self._pending = []

    # ------------------------------------------------------------------ reconstruction
    def reconstruction(self, file_hash: str, byte_range: tuple[int, int] | None = None) -> dict | None:
        f = self.file_index.get(file_hash)
        if f is None:
            return None
        # The server runs in the client's process (tests, bench.py's public-path row): its Python time
        # holds the GIL the measured pull needs, which a remote CAS would not.  A file's answer is
        # built once per term list (unpacked lengths from prefix sums) and re-served from the cache:
        # the 70B row's 30 answers cost 35 ms of GIL time per pull before (profiles/r6).
        ck = (file_hash, byte_range, id(f.terms), len(self.xorbs), self.xorb_url,
              self._srv.server_address if self._srv is not None else None)
        hit = self._recon_cache.get(ck)
        if hit is not None:
            return hit
        terms_out = []
        ranges: dict[int, list[list[int]]] = {}
        pos = 0
        offset_into_first = 0
        for (x, c0, c1) in f.terms:
            xb = self.xorbs[x]
            ulen = xb.cum[c1] - xb.cum[c0]
            t_start, t_end = pos, pos + ulen
            pos = t_end
            if byte_range is not None:
                a, b = byte_range
                if t_end <= a or t_start > b:
                    continue
                if not terms_out:
                    offset_into_first = max(0, a - t_start)
            terms_out.append({"hash": xb.hash_hex, "unpacked_length": ulen, "range": {"start": c0, "end": c1}})
            ranges.setdefault(x, []).append([c0, c1])
        # Like the real CAS: per xorb, one fetch entry per maximal union of the terms' chunk ranges,
        # so every term lies inside exactly one entry (hf_xet relies on this).
        fetch = {}
        for x, rs in ranges.items():
            rs.sort()
            merged = [rs[0][:]]
            for a, b in rs[1:]:
                if a <= merged[-1][1]:
                    merged[-1][1] = max(merged[-1][1], b)
                else:
                    merged.append([a, b])
            xb = self.xorbs[x]
            fetch[xb.hash_hex] = [{"range": {"start": a, "end": b}, "url": self._presign(xb.hash_hex),
                                   "url_range": {"start": xb.boundaries[a - 1] if a > 0 else 0,
                                                 "end": xb.boundaries[b - 1] - 1}} for a, b in merged]
        rec = {"offset_into_first_range": offset_into_first, "terms": terms_out, "fetch_info": fetch}
        self._recon_cache[ck] = rec
        return rec

    def _presign(self, hx: str) -> str:
        # Like S3 presigned URLs, the xorb URL carries its own authorization (clients such as hf_xet
        # fetch it without the CAS bearer token).
        if self.xorb_url:
            return f"{self.xorb_url}/{hx}"
        sig = hashlib.sha256(f"{self.token}:{hx}".encode()).hexdigest()[:32]
        return f"{self.url}/xorbs/default/{hx}?X-Zest-Signature={sig}"

    def _presign_ok(self, hx: str, query: dict) -> bool:
        want = hashlib.sha256(f"{self.token}:{hx}".encode()).hexdigest()[:32]
        return query.get("X-Zest-Signature", [""])[0] == want

    def file(self, repo_id: str, path: str, repo_type: str = "model") -> bytes:
        return self.repos[(repo_type, repo_id)].files[path].data

    def xet_hash(self, repo_id: str, path: str, repo_type: str = "model") -> str | None:
        return self.repos[(repo_type, repo_id)].files[path].xet_hash

    # ------------------------------------------------------------------ server
    @property
    def url(self) -> str:
        assert self._srv is not None, "FakeHub not started"
        return f"http://{self.host}:{self._srv.server_address[1]}"

    def start(self, port: int = 0) -> str:
        hub = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            disable_nagle_algorithm = True  # headers and body go out without waiting for ACKs

            def log_message(self, *a):  # quiet
                pass

            def do_GET(self):
                try:
                    hub._handle(self)
                except (BrokenPipeError, ConnectionResetError):
                    pass

            do_HEAD = do_GET

        class S(ThreadingHTTPServer):
            # socketserver's default listen backlog is 5: 16 concurrent reconstruction requests
            # (swarm_pull's plan) overflowed it and the dropped SYNs came back after the 1 s
            # retransmit -- the plan of a 70B pull took 1.06 s instead of ~0.1 (tools/plan_probe.py)
            request_queue_size = 1024

        self._srv = S((self.host, port), H)
        self._srv.daemon_threads = True
        self._thr = threading.Thread(target=self._srv.serve_forever, daemon=True)
        self._thr.start()
        return self.url

    def stop(self) -> None:
        if self._srv:
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None

    def __enter__(self):
        if self._srv is None:
            self.start()
        return self

    def __exit__(self, *exc):
        self.stop()

    def env(self, cache_root: str) -> dict[str, str]:
        """Environment for a client process pointed at this hub with caches under `cache_root`."""
        return {"HF_ENDPOINT": self.url, "HF_TOKEN": self.token, "HF_HOME": f"{cache_root}/hf",
                "HF_HUB_CACHE": f"{cache_root}/hf/hub", "ZEST_CACHE_DIR": f"{cache_root}/zest",
                "HOME": cache_root, "ZEST_NO_AUTOSTART": "1"}

    # ------------------------------------------------------------------ request handling
    def _count(self, k: str, n: int = 1) -> None:
        with self.lock:
            self.counters[k] = self.counters.get(k, 0) + n

    def _send(self, h, status: int, body: bytes, ctype: str = "application/json", headers: dict | None = None):
        h.send_response(status)
        h.send_header("Content-Type", ctype)
        h.send_header("Content-Length", str(len(body)))
        for k, v in (headers or {}).items():
            h.send_header(k, v)
        h.end_headers()
        if h.command != "HEAD":
            h.wfile.write(body)

    def _json(self, h, obj, status: int = 200, headers: dict | None = None):
        self._send(h, status, json.dumps(obj, separators=(",", ":")).encode(), headers=headers)

    def _authorized(self, h) -> bool:
        if not self.require_auth:
            return True
        return h.headers.get("Authorization", "") == f"Bearer {self.token}"

    def _cas_authorized(self, h) -> bool:
        return h.headers.get("Authorization", "") == f"Bearer xet-{self.token}"

    @staticmethod
    def _parse_range(h) -> tuple[int, int] | None:
        r = h.headers.get("Range")
        if not r or not r.startswith("bytes="):
            return None
        a, _, b = r[6:].partition("-")
        return int(a), (int(b) if b else 1 << 62)

    def _find_repo(self, kind: str, repo: str):
        return self.repos.get((kind, repo))

    def _handle(self, h) -> None:
        u = urllib.parse.urlsplit(h.path)
        path = urllib.parse.unquote(u.path)
        q = urllib.parse.parse_qs(u.query)
        parts = path.strip("/").split("/")
        self._count("requests")
        # ---- tracker
        if path == "/announce":
            return self._announce(h, u.query)
        # ---- CAS
        if parts[0] in ("v1", "v2") and len(parts) == 3 and parts[1] == "reconstructions":
            self._count(f"cas_{parts[0]}")
            if parts[0] == "v2":
                return self._json(h, {"error": "not found"}, 404)
            if not self._cas_authorized(h):
                return self._json(h, {"error": "unauthorized"}, 401)
            rng = self._parse_range(h)
            rec = self.reconstruction(parts[2], rng)
            if rec is None:
                return self._json(h, {"error": "file not found"}, 404)
            if rng is not None and not rec["terms"]:
                return self._json(h, {"error": "range not satisfiable"}, 416)
            return self._json(h, rec)
        if parts[0] == "reconstruction" and len(parts) == 2:
            return self._json(h, {"error": "not found"}, 404)
        if parts[0] == "xorbs" and len(parts) == 3:
            return self._xorb(h, parts[2], q)
        # ---- hub API
        if parts[0] == "api" and len(parts) >= 5 and parts[1] in ("models", "datasets", "spaces"):
            kind = parts[1][:-1]
            if not self._authorized(h):
                return self._json(h, {"error": "unauthorized"}, 401)
            # repo id is 1 or 2 path components: find the action keyword
            for i, p in enumerate(parts[2:], start=2):
                if p in ("tree", "revision", "xet-read-token"):
                    repo_id = "/".join(parts[2:i])
                    action, rest = p, parts[i + 1:]
                    break
            else:
                return self._json(h, {"error": "not found"}, 404)
            repo = self._find_repo(kind, repo_id)
            if repo is None:
                return self._json(h, {"error": "Repository not found"}, 404)
            rev = rest[0] if rest else "main"
            if rev not in repo.revisions:
                return self._json(h, {"error": "Revision not found"}, 404)
            if action == "revision":
                self._count("hub_revision")
                return self._json(h, {"id": repo.repo_id, "sha": repo.revisions[rev],
                                      "siblings": [{"rfilename": p} for p in repo.files]})
            if action == "xet-read-token":
                self._count("hub_token")
                return self._json(h, {"accessToken": f"xet-{self.token}", "casUrl": self.url,
                                      "exp": int(time.time()) + 3600})
            if action == "tree":
                self._count("hub_tree")
                entries = []
                for f in repo.files.values():
                    oid, sha = f.digests()
                    size = f.size if isinstance(f, _LazyFile) else len(f.data)
                    e = {"type": "file", "path": f.path, "size": size, "oid": oid}
                    if f.xet_hash:
                        e["xetHash"] = f.xet_hash
                        e["lfs"] = {"oid": sha, "size": size, "pointerSize": 134}
                    entries.append(e)
                entries.sort(key=lambda e: e["path"])
                start = int(q.get("cursor", ["0"])[0])
                headers = {}
                if self.page_size and start + self.page_size < len(entries):
                    nxt = dict((k, v[0]) for k, v in q.items())
                    nxt["cursor"] = str(start + self.page_size)
                    headers["Link"] = f'<{self.url}{u.path}?{urllib.parse.urlencode(nxt)}>; rel="next"'
                    entries = entries[start:start + self.page_size]
                elif self.page_size:
                    entries = entries[start:]
                return self._json(h, entries, headers=headers)
        # ---- /{repo}/resolve/{rev}/{path}
        if "resolve" in parts:
            i = parts.index("resolve")
            prefix = parts[:i]
            kind = "model"
            if prefix and prefix[0] in ("datasets", "spaces"):
                kind, prefix = prefix[0][:-1], prefix[1:]
            repo = self._find_repo(kind, "/".join(prefix))
            if repo is None or len(parts) < i + 3:
                return self._json(h, {"error": "not found"}, 404)
            rev, fpath = parts[i + 1], "/".join(parts[i + 2:])
            if rev not in repo.revisions or fpath not in repo.files:
                return self._json(h, {"error": "Entry not found"}, 404)
            if not self._authorized(h):
                return self._json(h, {"error": "unauthorized"}, 401)
            self._count("resolve")
            data = repo.files[fpath].data
            hdr = {"X-Repo-Commit": repo.revisions[rev], "ETag": f'"{repo.files[fpath].digests()[1]}"'}
            if repo.files[fpath].xet_hash:
                hdr["X-Xet-Hash"] = repo.files[fpath].xet_hash
            return self._send(h, 200, data, "application/octet-stream", hdr)
        return self._json(h, {"error": "not found"}, 404)

    def _xorb(self, h, hx: str, query: dict | None = None) -> None:
        if not self._cas_authorized(h) and not self._presign_ok(hx, query or {}):
            return self._json(h, {"error": "unauthorized"}, 401)
        idx = self.xorb_index.get(hx)
        if idx is None:
            return self._json(h, {"error": "xorb not found"}, 404)
        if hx in self.fail_xorbs:
            self._count("xorb_fail")
            return self._json(h, {"error": "injected failure"}, 500)
        if self.xorb_delay_s:
            with self._delay_lock:
                n = self._xorb_gets
                self._xorb_gets += 1
            time.sleep(self.xorb_delay_s * (1 + (n % self.xorb_delay_stagger if self.xorb_delay_stagger else 0)))
        data = self.xorbs[idx].data
        if data is None:  # metadata-only world: the bytes live with the peers
            self._count("xorb_missing")
            return self._json(h, {"error": "xorb payload not published"}, 404)
        rng = None if self.ignore_range else self._parse_range(h)
        status = 200
        if rng is not None:
            a, b = rng
            b = min(b, len(data) - 1)
            if a > b:
                return self._send(h, 416, b"", "application/octet-stream")
            data, status = data[a:b + 1], 206
        if hx in self.corrupt_xorbs and data:
            body = bytearray(data)
            body[len(body) // 2] ^= 0xFF
            data = bytes(body)
        self._count("xorb_get")
        with self.lock:
            self.xorb_bytes_served += len(data)
        self._send(h, status, data, "application/octet-stream")

    def _announce(self, h, query: str) -> None:
        # info_hash / peer_id are raw bytes percent-encoded: parse with latin-1 to keep them intact.
        q = urllib.parse.parse_qs(query, encoding="latin-1")
        try:
            ih = q["info_hash"][0].encode("latin-1")
            port = int(q["port"][0])
        except (KeyError, ValueError):
            return self._send(h, 200, _core.bencode.encode({"failure reason": "missing info_hash/port"}), "text/plain")
        self._count("announce")
        ip = h.client_address[0]
        now = time.time()
        with self.lock:
            swarm = self.tracker_peers.setdefault(ih, {})
            me = f"{ip}:{port}"
            if q.get("event", [""])[0] == "stopped":
                swarm.pop(me, None)
            else:
                swarm[me] = now
            peers = [p for p in swarm if p != me]
        compact = b"".join(_core.tracker.encode_compact_peer(p) for p in peers)
        self._send(h, 200, _core.bencode.encode({"interval": 60, "peers": compact}), "text/plain")


def main(argv=None) -> int:
    """`python -m zest_amd.testing.fakehub`: serve a directory or a synthetic model as an offline Hub.

    Prints one JSON line {"url", "token", "repo", "commit", "tracker"} and serves until SIGTERM /
    Ctrl-C (scripts/p2p_cluster_test.sh uses it for air-gapped runs)."""
    import argparse
    import os
    import signal

    ap = argparse.ArgumentParser(prog="python -m zest_amd.testing.fakehub")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--repo", default="zest-test/model")
    ap.add_argument("--dir", help="publish the files under this directory as --repo")
    ap.add_argument("--model", default="llama-tiny", help="synthetic model spec (zest_amd.models) when --dir is absent")
    ap.add_argument("--policy", default="auto", choices=["none", "lz4", "bg4", "auto"])
    ap.add_argument("--max-xorb-bytes", type=int, default=64 << 20)
    a = ap.parse_args(argv)
    hub = FakeHub(policy=a.policy, max_xorb_bytes=a.max_xorb_bytes)
    if a.dir:
        files = {}
        for root, _, names in os.walk(a.dir):
            for n in names:
                p = os.path.join(root, n)
                with open(p, "rb") as fh:
                    files[os.path.relpath(p, a.dir)] = fh.read()
        commit = hub.add_repo(a.repo, files)
        repo = a.repo
    else:
        from .. import models
        from ..synthetic import SyntheticWorld

        world = SyntheticWorld(models.get(a.model), seed=0, max_xorb_bytes=a.max_xorb_bytes)
        commit = hub.add_world(world)
        repo = world.spec.repo_id
    hub.host = a.host
    url = hub.start(a.port)
    print(json.dumps({"url": url, "token": hub.token, "repo": repo, "commit": commit, "tracker": f"{url}/announce"}),
          flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    try:
        while not stop.wait(1.0):
            pass
    except KeyboardInterrupt:
        pass
    hub.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
