#!/bin/bash
# round 5 (an): rocprofv3 kernel trace + FETCH/WRITE/L2 passes of the final tree per config (C5:
# profiles/r05al_c5/), for the final numbers in DESIGN.md 5.3
set -o pipefail
O=gpurun_out/r05an
mkdir -p $O
for cfg in c3 c3s c4 c3t; do
  timeout -k 10 600 bash profiles/run_profiles.sh r05an_$cfg --config $cfg > $O/prof_$cfg.log 2>&1 || exit 1
done
timeout -k 10 600 bash profiles/run_profiles.sh r05an_c3b1 --config c3 --batch 1 > $O/prof_c3b1.log 2>&1 || exit 1
