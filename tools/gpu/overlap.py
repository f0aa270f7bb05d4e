"""Copy/compute overlap from a rocprofv3 --kernel-trace --memory-copy-trace CSV run.

    python tools/gpu/overlap.py OUT_DIR [--kernel ingest|place|lz4|hash] [--after-s 0]

Reports, over the time window spanned by host->device copies (optionally only the part after
`--after-s` seconds from the first event): H2D busy seconds, matching-kernel busy seconds, the time
both were active at once, and the H2D bytes / GB/s -- the evidence that a pipeline's PCIe copies
run under its decode/hash kernels instead of in series with them.
"""
import argparse
import csv
import glob
import os


def intervals(rows, key_start="Start_Timestamp", key_end="End_Timestamp"):
    return sorted((float(r[key_start]), float(r[key_end])) for r in rows)


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def total(u):
    return sum(b - a for a, b in u)


def inter(u1, u2):
    i = j = 0
    s = 0.0
    while i < len(u1) and j < len(u2):
        a, b = max(u1[i][0], u2[j][0]), min(u1[i][1], u2[j][1])
        if b > a:
            s += b - a
        if u1[i][1] < u2[j][1]:
            i += 1
        else:
            j += 1
    return s


def from_db(out):
    """(kernel rows, copy rows) as CSV-like dicts from a rocpd SQLite database (rocprofv3's default
    output), or None when there is none."""
    import sqlite3
    dbs = glob.glob(os.path.join(out, "**", "*.db"), recursive=True)
    if not dbs:
        return None
    c = sqlite3.connect(dbs[0])

    def cols(view):
        return [r[1] for r in c.execute(f"pragma table_info({view})").fetchall()]

    def pick(cs, *names):
        return next((n for n in names if n in cs), None)
    kc, mc = cols("kernels"), cols("memory_copies")
    ks, ke, kn = pick(kc, "start", "start_ns"), pick(kc, "end", "end_ns"), pick(kc, "name", "kernel_name")
    kt = [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b}
          for n, a, b in c.execute(f"select {kn}, {ks}, {ke} from kernels").fetchall()]
    ms, me = pick(mc, "start", "start_ns"), pick(mc, "end", "end_ns")
    mn, mz = pick(mc, "name", "direction", "kind"), pick(mc, "size", "bytes")
    cp = [{"Direction": n, "Start_Timestamp": a, "End_Timestamp": b, "Size": z}
          for n, a, b, z in c.execute(f"select {mn}, {ms}, {me}, {mz} from memory_copies").fetchall()]
    print(f"rocpd db {os.path.basename(dbs[0])}: kernel columns {kc[:12]}...; copy columns {mc}")
    return kt, cp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--kernel", default="ingest,place,lz4,hash,blake3,decode")
    ap.add_argument("--after-s", type=float, default=0.0)
    ap.add_argument("--marker", default="", help="restrict to the roctx range whose record contains this text")
    ap.add_argument("--between", default="", help="restrict to the span between the first and last launch of "
                                                 "kernels whose name contains this text")
    a = ap.parse_args()
    db = from_db(a.out)
    if db is not None:
        kt, mc = db
    else:
        kt = [r for f in glob.glob(os.path.join(a.out, "**", "*kernel_trace.csv"), recursive=True)
              for r in csv.DictReader(open(f))]
        mc = [r for f in glob.glob(os.path.join(a.out, "**", "*memory_copy_trace.csv"), recursive=True)
              for r in csv.DictReader(open(f))]
    h2d = [r for r in mc if "HOST_TO_DEVICE" in (r.get("Direction", "") + r.get("Operation", "")).upper()]
    pats = [p for p in a.kernel.split(",") if p]
    ks = [r for r in kt if any(p in r.get("Kernel_Name", "").lower() for p in pats)]
    t0 = min(float(r["Start_Timestamp"]) for r in kt + mc) if (kt or mc) else 0.0
    lo, hi = t0 + a.after_s * 1e9, float("inf")
    if a.marker:
        mk = [r for f in glob.glob(os.path.join(a.out, "**", "*marker_api_trace.csv"), recursive=True)
              for r in csv.DictReader(open(f)) if any(a.marker in str(v) for v in r.values())]
        if not mk:
            raise SystemExit(f"no roctx range containing {a.marker!r}")
        lo, hi = min(float(r["Start_Timestamp"]) for r in mk), max(float(r["End_Timestamp"]) for r in mk)
        print(f"marker {a.marker!r}: {(hi - lo) / 1e9:.3f} s")
    if a.between:
        mk = [r for r in kt if a.between in r.get("Kernel_Name", "")]
        if len(mk) < 2:
            raise SystemExit(f"fewer than two kernels named *{a.between}*")
        lo, hi = min(float(r["End_Timestamp"]) for r in mk), max(float(r["Start_Timestamp"]) for r in mk)
        print(f"between {a.between!r} kernels: {(hi - lo) / 1e9:.3f} s")
    h2d = [r for r in h2d if lo <= float(r["Start_Timestamp"]) <= hi]
    ks = [r for r in ks if lo <= float(r["Start_Timestamp"]) <= hi]
    if mc:
        print("memory copy columns:", list(mc[0].keys()))
    uh, uk = union(intervals(h2d)), union(intervals(ks))
    size_key = next((k for k in (h2d[0].keys() if h2d else []) if k.lower() in ("size", "bytes", "copy_bytes")), None)
    nbytes = sum(float(r.get(size_key, 0) or 0) for r in h2d) if size_key else 0.0
    span = (max(b for _, b in uh) - min(a_ for a_, _ in uh)) / 1e9 if uh else 0.0
    both = inter(uh, uk) / 1e9
    print(f"window {span:.3f} s (H2D first..last): H2D busy {total(uh) / 1e9:.3f} s, "
          f"{nbytes / 1e9:.2f} GB -> {nbytes / max(1e-9, total(uh) / 1e9) / 1e9:.1f} GB/s while busy, "
          f"{nbytes / max(1e-9, span) / 1e9:.1f} GB/s over the window")
    print(f"kernels matching {pats}: busy {total(uk) / 1e9:.3f} s; concurrent with H2D {both:.3f} s "
          f"({100 * both / max(1e-9, total(uk) / 1e9):.0f} % of kernel time, "
          f"{100 * both / max(1e-9, total(uh) / 1e9):.0f} % of H2D time)")


if __name__ == "__main__":
    main()
