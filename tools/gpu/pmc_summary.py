"""Per-kernel sums of a rocprofv3 --pmc counter_collection.csv (tools/gpu/check.sh kpmc step).

    python tools/gpu/pmc_summary.py <counter_collection.csv> [kernel-substring]
"""
import collections
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for r in rows:
        k = r.get("Kernel_Name", "")
        if want and want not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for k, d in sorted(agg.items()):
        n = max(1, len(launches[k]))
        print(f"{k[:60]}  launches={n}  " + "  ".join(f"{c}={v / n:.4g}" for c, v in sorted(d.items())))


if __name__ == "__main__":
    main()
