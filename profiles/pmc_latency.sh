#!/bin/bash
# profiles/pmc_latency.sh TAG: address/TLB/latency counters of k_render at C3, one rocprofv3
# --pmc pass per group (block limits: 2 TA, 2 TD, 4 TCP, 2 GRBM), per-dispatch means into
# $OUT/table.txt (profiles/pmc_table.py).
set -euo pipefail
TAG=${1:?tag}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmclat_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
GROUPS_=("TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE GRBM_TA_BUSY"
         "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ"
         "TCP_TCP_TA_DATA_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES")
i=0
for G in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G --output-format csv -d "$OUT/g$i" -o run \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$OUT/g$i.json" 2> "$OUT/g$i.err"
done
python3 "$ROOT/profiles/pmc_table.py" "$OUT" "g" > "$OUT/table.txt"
cat "$OUT/table.txt"
