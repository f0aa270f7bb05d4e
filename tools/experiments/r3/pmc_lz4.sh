export ZEST_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r3v
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAVES --kernel-trace -d gpurun_out/r3v/pmc -o p1 --output-format csv -- python3 tools/kbench.py --only lz4occ > gpurun_out/r3v/p1.log 2>&1 || { tail -20 gpurun_out/r3v/p1.log; exit 1; }
f=$(find gpurun_out/r3v/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", "")[:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "lz4" in k:
        print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
rm -rf gpurun_out/r3v/pmc
