"""Per-kernel counter table from several rocprofv3 --pmc passes (tools/gpu/check.sh pmctable step).

    python tools/gpu/pmc_table.py OUT_DIR/pmc_A OUT_DIR/pmc_B ... > table.md

Each pass directory holds a counter_collection.csv (per-dispatch counters) and a kernel_trace.csv
(per-dispatch start/end).  For every kernel: launches, mean duration, HBM bytes read / written per
launch (FETCH_SIZE / WRITE_SIZE are KiB in rocprof's definition) and the achieved GB/s, VALU busy and
utilization (active lanes / 64), the fraction of wave-cycles issuing VALU / SALU instructions,
LDS bank-conflict ratio, FLAT and VMEM instruction counts, wait fraction.  Round 4's pass used
SQ_ACTIVE_INST_VMEM, which reads 0 on gfx950 for kernels that stream GBs through global_* loads;
SQ_INSTS_VMEM / SQ_INSTS_FLAT count them.  Raw per-kernel counter means go to `--raw FILE` (JSON).
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            dur[k].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)  # us
    return cnt, disp, dur


def short(k):
    k = k.replace("(anonymous namespace)::", "")
    return k.split("(")[0][:34]


def main():
    raw = None
    if "--raw" in sys.argv:
        i = sys.argv.index("--raw")
        raw = sys.argv[i + 1]
        del sys.argv[i:i + 2]
    per = collections.defaultdict(dict)
    launches, durs = {}, collections.defaultdict(list)
    for d in sys.argv[1:]:
        cnt, disp, dur = load(d)
        for k, c in cnt.items():
            n = max(1, len(disp[k]))
            launches[k] = max(launches.get(k, 0), n)
            for name, v in c.items():
                per[k][name] = v / n
        for k, v in dur.items():
            durs[k] += v
    rows = []
    for k in per:
        c = per[k]
        us = sum(durs[k]) / len(durs[k]) if durs[k] else 0.0
        rd = c.get("FETCH_SIZE", 0) * 1024
        wr = c.get("WRITE_SIZE", 0) * 1024
        gbps = (rd + wr) / (us * 1e3) if us else 0.0
        act = c.get("SQ_ACTIVE_INST_VALU", 0)
        util = 100 * c.get("SQ_THREAD_CYCLES_VALU", 0) / (act * 64) if act else 0.0
        wcyc = c.get("SQ_WAVE_CYCLES", 0)
        # per-wave issue fractions (independent of how rocprof sums SE / XCD instances)
        valu_busy = 100 * act / wcyc if wcyc else 0.0
        salu_busy = 100 * c.get("SQ_ACTIVE_INST_SCA", 0) / wcyc if wcyc else 0.0
        lds_act = c.get("SQ_LDS_IDX_ACTIVE", 0) - c.get("SQ_LDS_BANK_CONFLICT", 0)
        bank = c.get("SQ_LDS_BANK_CONFLICT", 0) / lds_act if lds_act > 0 else 0.0
        wait = 100 * c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else 0.0
        rows.append((us * launches[k], short(k), launches[k], us, rd / 1e6, wr / 1e6, gbps, valu_busy, util, salu_busy,
                     bank, c.get("SQ_INSTS_FLAT", 0), c.get("SQ_INSTS_VMEM", 0), c.get("SQ_INSTS_LDS", 0), wait))
    rows.sort(reverse=True)
    if raw:
        import json
        with open(raw, "w") as f:
            json.dump({k: dict(v) for k, v in per.items()}, f, indent=1)
    print("| kernel | launches | us/launch | HBM rd MB | HBM wr MB | GB/s | VALU issue % of wave-cycles | "
          "VALU util % | SALU issue % of wave-cycles | LDS conflict/access | FLAT insts | VMEM insts | LDS insts | "
          "wait-inst % |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        print(f"| {r[1]} | {r[2]} | {r[3]:.1f} | {r[4]:.1f} | {r[5]:.1f} | {r[6]:.0f} | {r[7]:.1f} | {r[8]:.1f} | "
              f"{r[9]:.1f} | {r[10]:.3f} | {r[11]:.3g} | {r[12]:.3g} | {r[13]:.3g} | {r[14]:.1f} |")


if __name__ == "__main__":
    main()
