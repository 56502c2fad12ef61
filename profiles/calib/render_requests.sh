#!/bin/bash
# profiles/calib/render_requests.sh CONFIG: the render kernel's L2->fabric read requests by
# size (64 B / 128 B) and those that went to DRAM (not served by the Infinity Cache), over
# the same bench.py run as run_profiles.sh; per-launch means of k_render.
set -euo pipefail
CFG=${1:-c3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/req_$CFG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum \
  --output-format csv -d "$OUT/req" -o run -- python3 "$ROOT/bench.py" --config "$CFG" --steps 20 --warmup 2 --no-cpu-baseline --no-single-compare \
  > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_sum \
  --output-format csv -d "$OUT/wr" -o run -- python3 "$ROOT/bench.py" --config "$CFG" --steps 20 --warmup 2 --no-cpu-baseline --no-single-compare \
  > /dev/null 2>> "$OUT/bench.err" || echo "write-request pass failed" >&2
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_render" not in r["Kernel_Name"]:
            continue
        if int(r.get("Grid_Size", 0) or 0) <= int(r.get("Workgroup_Size", 0) or 0):
            continue  # the context's one-workgroup prewarm dispatch
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, c in per.items():
        for k, v in c.items():
            acc[k].append(v)
res = {k: sum(v) / len(v) for k, v in acc.items()}
rd64, rd128 = res.get("TCC_EA0_RDREQ_64B_sum", 0), res.get("TCC_EA0_RDREQ_128B_sum", 0)
res["read_bytes_per_launch"] = 64 * rd64 + 128 * rd128
print(json.dumps(res, indent=1))
PY
