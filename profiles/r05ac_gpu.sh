#!/bin/bash
# round 5 (ac): the slot table built by default only when the headers outgrow the last-level cache
# (C5) -- the whole GPU suite, smoke, the default bench line and C5's
set -o pipefail
O=gpurun_out/${RUN:-r05ac}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_c3_full.json 2> $O/bench_c3_full.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
