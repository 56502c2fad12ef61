#!/bin/bash
# profiles/pmc_pass.sh OUTDIR "COUNTERS..." [ab_variants args]: one rocprofv3 --pmc pass
# over profiles/ab_variants.py (kernel-trace only besides the counters).
set -euo pipefail
OUT=$1; shift
CNT=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d "$ROOT/gpurun_out/$OUT" -o run \
  -- python3 "$ROOT/profiles/ab_variants.py" "$@" > "$ROOT/gpurun_out/$OUT/ab.jsonl" 2> "$ROOT/gpurun_out/$OUT/ab.err"
