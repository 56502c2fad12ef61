# round 3 (zh): every scene on the 5-wave default (the 4-wave footprint rule removed): full GPU
# suite (C5 whole frame now at 5 waves), smoke, the default bench line, rocprofv3 stats + PMC
# at C5 and C3
set -o pipefail
mkdir -p gpurun_out/r03zh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03zh/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zh/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03zh/bench.json 2> gpurun_out/r03zh/bench.err || exit 1
bash profiles/run_profiles.sh r03zh_c5 --config c5 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03zh_c3 --config c3 > /dev/null 2>&1 || exit 1
