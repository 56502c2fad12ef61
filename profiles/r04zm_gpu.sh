# round 4 (zm): the final tree once more -- smoke, the full GPU suite, the default bench
set -o pipefail
O=gpurun_out/r04zm
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
