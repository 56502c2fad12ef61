#!/bin/bash
# round 6 (ze): the final tree's C5 (quad slot table, the most sub-cells' first candidate as the copy):
# rocprofv3 kernel trace + FETCH/WRITE/L2 passes, then the default bench line with its secondary block
set -o pipefail
O=gpurun_out/r06ze
mkdir -p $O
timeout -k 10 700 bash profiles/run_profiles.sh r06ze_c5 --config c5 > $O/prof_c5.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
