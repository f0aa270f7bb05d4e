"""Per-copy H2D rates from a rocprofv3 --kernel-trace --memory-copy-trace run (rocpd database), split
into the engine part and the public-path part of a bench run (the public-path swarm row is bracketed
by `spin_kernel` launches under ZEST_BENCH_MARK=1), and by how much of each copy ran under a decode /
hash kernel.

    python tools/gpu/copy_rates.py OUT_DIR [--min-mb 256] [--between spin_kernel]

Question it answers: does an H2D copy run slower while the LZ4 decoder (or any other kernel) runs?
Copies are bucketed by the fraction of their duration that overlapped a kernel matching --kernel.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from overlap import from_db, union  # noqa: E402


def overlap_frac(a, b, ku):
    """Fraction of [a, b) covered by the union ku (sorted, disjoint)."""
    s = 0.0
    for x, y in ku:
        if y <= a:
            continue
        if x >= b:
            break
        s += min(b, y) - max(a, x)
    return s / max(1.0, b - a)


def report(tag, copies, kernels, pats, min_bytes):
    big = [r for r in copies if float(r["Size"] or 0) >= min_bytes]
    if not big:
        print(f"[{tag}] no H2D copies >= {min_bytes >> 20} MiB")
        return
    ks = [r for r in kernels if any(p in r["Kernel_Name"].lower() for p in pats)]
    ku = union([(float(r["Start_Timestamp"]), float(r["End_Timestamp"])) for r in ks])
    rows = []
    for r in big:
        a, b, z = float(r["Start_Timestamp"]), float(r["End_Timestamp"]), float(r["Size"])
        rows.append((z / max(1.0, b - a), overlap_frac(a, b, ku), z, b - a))
    tot_b = sum(r[2] for r in rows)
    tot_t = sum(r[3] for r in rows)
    print(f"[{tag}] {len(rows)} H2D copies >= {min_bytes >> 20} MiB: {tot_b / 1e9:.2f} GB, "
          f"{tot_b / tot_t:.1f} GB/s over their busy time")
    for lo, hi in ((0.0, 0.1), (0.1, 0.5), (0.5, 0.9), (0.9, 1.01)):
        sel = [r for r in rows if lo <= r[1] < hi]
        if sel:
            b = sum(r[2] for r in sel)
            t = sum(r[3] for r in sel)
            print(f"  overlap with {pats} in [{lo:.1f}, {min(hi, 1.0):.1f}): {len(sel)} copies, {b / t:.1f} GB/s")
    # every kernel name active in the window, by total time (a blit-kernel copy would show here)
    a0 = min(float(r["Start_Timestamp"]) for r in big)
    b0 = max(float(r["End_Timestamp"]) for r in big)
    agg: dict = {}
    for r in kernels:
        s = float(r["Start_Timestamp"])
        if a0 <= s <= b0:
            n = r["Kernel_Name"].split("(")[0][:60]
            c, t = agg.get(n, (0, 0.0))
            agg[n] = (c + 1, t + float(r["End_Timestamp"]) - s)
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]:
        print(f"  kernel {n}: {c} launches, {t / 1e6:.1f} ms")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--min-mb", type=int, default=256)
    ap.add_argument("--kernel", default="lz4,ingest,hash,blake3,place")
    ap.add_argument("--between", default="spin_kernel")
    a = ap.parse_args()
    db = from_db(a.out)
    if db is None:
        raise SystemExit("no rocpd database under " + a.out)
    kt, mc = db
    h2d = [r for r in mc if "HOST_TO_DEVICE" in str(r["Direction"]).upper()]
    pats = [p for p in a.kernel.split(",") if p]
    mk = sorted(float(r["Start_Timestamp"]) for r in kt if a.between and a.between in r["Kernel_Name"])
    if len(mk) >= 2:
        lo, hi = mk[0], mk[-1]
        inside = [r for r in h2d if lo <= float(r["Start_Timestamp"]) <= hi]
        outside = [r for r in h2d if not lo <= float(r["Start_Timestamp"]) <= hi]
        report("engine (outside the spin-kernel brackets)", outside, kt, pats, a.min_mb << 20)
        report("public path (between the spin kernels)", inside, kt, pats, a.min_mb << 20)
    else:
        report("all", h2d, kt, pats, a.min_mb << 20)


if __name__ == "__main__":
    main()
