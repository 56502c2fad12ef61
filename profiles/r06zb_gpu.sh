#!/bin/bash
# round 6 (zb): rocprofv3 kernel trace + FETCH/WRITE/L2 passes of the final tree per config (DESIGN.md
# 5.3 and the bench line's traffic): C3 8 chained frames, C3 one launch per frame, C3t, C3s, C4,
# C5 (quad slot table)
set -o pipefail
O=gpurun_out/r06zb
mkdir -p $O
for cfg in c3 c3t c3s c4 c5; do
  timeout -k 10 700 bash profiles/run_profiles.sh r06zb_$cfg --config $cfg > $O/prof_$cfg.log 2>&1 || exit 1
done
timeout -k 10 600 bash profiles/run_profiles.sh r06zb_c3b1 --config c3 --batch 1 > $O/prof_c3b1.log 2>&1 || exit 1
