"""GPU activity inside the public-path row's timed window of a multi-rank rehearsal (every rank's
process traced: rocprofv3 --kernel-trace --memory-copy-trace --output-format csv, bench.py run with
ZEST_BENCH_MARK=1 so each rank brackets its timed calls with a sleep kernel).

    python tools/gpu/row_window.py OUT_DIR

Per rank the window runs from the end of its first marker kernel to the start of its second; the
report covers the span from the earliest window start to the latest window end: the union of every
process's kernels (how much of the span the GPU was running anything), the kernels by name (summed
and union time), and the host->device / device->device copies (union time and bytes).
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from overlap import inter, total, union  # noqa: E402


def main() -> int:
    d = sys.argv[1]
    kfiles = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    windows, kernels = [], []
    for f in kfiles:
        rows = list(csv.DictReader(open(f)))
        marks = sorted((float(r["Start_Timestamp"]), float(r["End_Timestamp"])) for r in rows
                       if "spin" in r["Kernel_Name"] or "sleep" in r["Kernel_Name"].lower())
        if len(marks) >= 2:
            windows.append((marks[0][1], marks[1][0]))
        kernels += [(float(r["Start_Timestamp"]), float(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48])
                    for r in rows]
    if not windows:
        print("no marker kernels found")
        return 1
    w0, w1 = min(a for a, _ in windows), max(b for _, b in windows)
    span = (w1 - w0) / 1e9
    ins = [(max(a, w0), min(b, w1), n) for a, b, n in kernels if b > w0 and a < w1]
    ku = union([(a, b) for a, b, _ in ins])
    by = collections.defaultdict(list)
    for a, b, n in ins:
        by[n].append((a, b))
    print(f"ranks with a window: {len(windows)}; span {span * 1e3:.1f} ms "
          f"(per-rank windows {min((b - a) for a, b in windows) / 1e6:.1f}-{max((b - a) for a, b in windows) / 1e6:.1f} ms)")
    print(f"GPU running any kernel: {total(ku) / 1e6:.1f} ms ({100 * total(ku) / (w1 - w0):.1f} % of the span)")
    rows = sorted(((sum(b - a for a, b in iv), total(union(iv)), len(iv), n) for n, iv in by.items()), reverse=True)
    print("| kernel | launches | summed ms | union ms |")
    print("|---|---:|---:|---:|")
    for s, u, c, n in rows[:14]:
        print(f"| `{n}` | {c} | {s / 1e6:.1f} | {u / 1e6:.1f} |")
    cfiles = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    cp = collections.defaultdict(list)
    nbytes = collections.Counter()
    for f in cfiles:
        for r in csv.DictReader(open(f)):
            a, b = float(r["Start_Timestamp"]), float(r["End_Timestamp"])
            if b <= w0 or a >= w1:
                continue
            kind = r.get("Direction", r.get("Operation", "?"))
            cp[kind].append((max(a, w0), min(b, w1)))
            nbytes[kind] += int(float(r.get("Size", r.get("Bytes", 0)) or 0))
    for kind, iv in cp.items():
        u = union(iv)
        print(f"copies {kind}: {len(iv)}, union {total(u) / 1e6:.1f} ms, {nbytes[kind] / 1e9:.2f} GB, "
              f"under kernels {inter(u, ku) / 1e6:.1f} ms")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
