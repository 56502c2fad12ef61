#!/bin/bash
# round 6 (zh): scenes with holes run the located-mode void walk by default (OPT_VOIDLOC): the whole GPU
# suite, the smoke frame, C3t's rocprofv3 + PMC passes (its kernel is now k_render<1147143456>) and
# the default bench line
set -o pipefail
O=gpurun_out/r06zh
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 bash profiles/run_profiles.sh r06zh_c3t --config c3t > $O/prof_c3t.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
