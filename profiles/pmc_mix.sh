#!/bin/bash
# profiles/pmc_mix.sh OUT LIB... : one rocprofv3 --pmc pass per library (IRT_LIB_PATH) with
# the SQ instruction-mix counters over a bench run (C3, or $CONFIG); prints per-wave averages for k_render.
set -uo pipefail
OUT=${1:?out}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  IRT_LIB_PATH="$ROOT/$lib" timeout -s KILL 120 rocprofv3 --kernel-trace \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$ROOT/$OUT/$n" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --config ${CONFIG:-c3} \
    > "$ROOT/$OUT/$n.json" 2> "$ROOT/$OUT/$n.err" || exit 1
done
python3 - "$ROOT/$OUT" <<'PY'
import csv, glob, os, sys, collections
root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*/"))):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_render" in row.get("Kernel_Name", ""):
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    # each dispatch's value per counter is the sum over its rows (dimensions)
    tot = {k: sum(v) for k, v in acc.items()}
    waves = tot.get("SQ_WAVES", 0) or 1
    print(os.path.basename(d.rstrip("/")), {k: round(v / waves, 1) for k, v in sorted(tot.items())})
PY
