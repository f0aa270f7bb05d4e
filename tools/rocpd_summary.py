"""Summarize a rocprofv3 SQLite (rocpd) database: per-kernel and per-copy totals.

    python tools/rocpd_summary.py gpurun_out/prof/bench8b_results.db > profiles/bench8b_kernels.md

rocprofv3 on ROCm 7 writes `<name>_results.db` by default; the `top_kernels` view reports
durations in microseconds.
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:70]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--title", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    print(f"# rocprofv3 kernel summary: {a.title or a.db}\n")
    print("| kernel | calls | total ms | avg us | % GPU time | grid | block | VGPR | LDS B |")
    print("|---|---:|---:|---:|---:|---|---|---:|---:|")
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), max(grid_x), max(workgroup_x), max(vgpr_count), "
        "max(lds_size) from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    for name, n, s, avg, gx, wx, vg, lds in rows:
        print(f"| `{short(name)}` | {n} | {s / 1e6:.3f} | {avg / 1e3:.1f} | {100 * s / tot:.1f} | {gx} | {wx} | {vg} | {lds} |")
    print(f"\nTotal kernel time: {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches.\n")
    try:
        cp = c.execute("select name, count(*), sum(size), sum(duration) from memory_copies group by name").fetchall()
        if cp:
            print("| copy | count | GiB | ms | GB/s |")
            print("|---|---:|---:|---:|---:|")
            for name, n, size, dur in cp:
                gbps = size / dur if dur else 0
                print(f"| {name} | {n} | {size / 2**30:.2f} | {dur / 1e6:.2f} | {gbps:.1f} |")
    except sqlite3.Error:
        pass


if __name__ == "__main__":
    main()
