#!/bin/bash
# round 6 (zp): the final tree (the TF statistic's buffer kept by the context): the whole GPU suite,
# smoke, bench
set -o pipefail
O=gpurun_out/r06zp
mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 450 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
