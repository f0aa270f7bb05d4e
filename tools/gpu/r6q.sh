# round-6 call q: host striping from 1 vs 3 uncapped loopback seeders (8 GB repo), leecher
# concurrency 16 vs 48; per-phase span totals and each seeder's lookup / send seconds
set -o pipefail
export TMPDIR=/tmp
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)  nproc: $(nproc)  tmp: $(df -h /tmp | tail -1)"
STRIPE_MB=8192 bash tools/gpu/check.sh r6q_j16 stripe && \
STRIPE_MB=8192 STRIPE_ARGS="--jobs 48" bash tools/gpu/check.sh r6q_j48 stripe && \
python - <<'PY'
import json
for t in ("r6q_j16", "r6q_j48"):
    d = json.load(open(f"gpurun_out/{t}/stripe.json"))
    print(t, "speedup", d["speedup_3_vs_1"], "transfer", d.get("transfer_speedup_3_vs_1"))
    for k in ("1_seeder", "3_seeders"):
        print(" ", k, {x: d[k][x] for x in ("seconds", "GBps", "transfer_s", "seeders") if x in d[k]})
        print("    spans", d[k].get("span_ms"))
PY
