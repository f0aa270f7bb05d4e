#!/usr/bin/env python3
"""Aggregate a ZEST_TRACE Chrome trace: per (category, span) count, summed and mean duration, and
the trace's wall span, and for each span how many threads ran it and how many of those are fetch
threads (threads that issue peer requests or CDN fetches).  `python tools/trace_summary.py trace.json [--top 25]`"""
from __future__ import annotations

import argparse
import collections
import json


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ev = json.load(open(a.trace))
    ev = ev["traceEvents"] if isinstance(ev, dict) else ev
    agg = collections.defaultdict(lambda: [0, 0.0])
    tids = collections.defaultdict(set)  # (cat, name) -> threads that ran it
    span = {}  # (cat, name) -> [first start, last end] in us
    ts = []
    threads = set()
    for e in ev:
        if e.get("ph") != "X":
            continue
        k = (e.get("cat", ""), e.get("name", ""))
        agg[k][0] += 1
        agg[k][1] += e.get("dur", 0) / 1e3
        ts += [e["ts"], e["ts"] + e.get("dur", 0)]
        lo, hi = span.get(k, (e["ts"], e["ts"] + e.get("dur", 0)))
        span[k] = (min(lo, e["ts"]), max(hi, e["ts"] + e.get("dur", 0)))
        threads.add(e.get("tid"))
        tids[k].add(e.get("tid"))
    wall = (max(ts) - min(ts)) / 1e3 if ts else 0.0
    print(f"wall span {wall:.1f} ms, {len(threads)} threads")
    t0 = min(ts) if ts else 0
    # fetch threads: the ones that issue peer requests or CDN fetches (the pull's network workers)
    fetch = set()
    for (c, n), ts_ in tids.items():
        if (c == "peer" and n == "request") or c == "cdn":
            fetch |= ts_
    print(f"{'category':10s} {'span':34s} {'count':>7s} {'sum ms':>10s} {'mean ms':>9s} {'first..last ms':>16s} "
          f"{'threads':>7s} {'on fetch thr':>12s}")
    for (c, n), (cnt, ms) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        lo, hi = span[(c, n)]
        print(f"{c:10s} {n:34s} {cnt:7d} {ms:10.1f} {ms / cnt:9.2f} {(lo - t0) / 1e3:7.1f}..{(hi - t0) / 1e3:<7.1f} "
              f"{len(tids[(c, n)]):7d} {len(tids[(c, n)] & fetch):12d}")


if __name__ == "__main__":
    main()
