#!/bin/bash
# round 6 (za): the final tree (fresh_args everywhere, slot units, split threshold 0.35 on scenes with
# holes): the whole GPU suite, the smoke frame and the default bench line
set -o pipefail
O=gpurun_out/r06za
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
