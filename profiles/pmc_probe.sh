#!/bin/bash
# profiles/pmc_probe.sh TAG "CASE1;CASE2;..." : for each probe.py case (C3) and each counter
# group, one rocprofv3 --pmc pass (counters never combined with traces); per-dispatch means
# of k_render in $OUT/table.txt.
set -euo pipefail
TAG=${1:?tag}
CASES=${2:?cases}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
         "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH"
         "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM")
IFS=';' read -ra CS <<< "$CASES"
j=0
for C in "${CS[@]}"; do
  j=$((j+1))
  i=0
  for G in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G --output-format csv -d "$OUT/c${j}_g$i" -o run \
      -- python3 "$ROOT/profiles/probe.py" --config c3 --rounds 1 --frames 3 --cases "$C" \
      > "$OUT/c${j}_g$i.jsonl" 2> "$OUT/c${j}_g$i.err"
  done
  echo "case $j: $C" >> "$OUT/table.txt"
  python3 "$ROOT/profiles/pmc_table.py" "$OUT" "c${j}_" >> "$OUT/table.txt"
done
cat "$OUT/table.txt"
