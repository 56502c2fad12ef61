#!/bin/bash
# profiles/calib/run.sh: FETCH_SIZE and TCC_EA0_RDREQ per calibration kernel (GPU box)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/calib
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- "$ROOT/profiles/calib/fetch_calibration" > "$OUT/run.json"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d "$OUT/req" -o run \
  -- "$ROOT/profiles/calib/fetch_calibration" > /dev/null || echo "request-counter pass failed" >&2
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
res = {}
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_gather" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("<")[1].split(">")[0]
        res.setdefault(k, {})[r["Counter_Name"]] = res.setdefault(k, {}).get(r["Counter_Name"], 0) + float(r["Counter_Value"])
print(json.dumps(res, indent=1))
PY
