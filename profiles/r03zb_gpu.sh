# round 3 (zb): streaming (nt) pixel stores as the default -- full GPU suite + smoke on it, A/B
# against the previous default (abl/lib_evdt.so) and an nt accum prefetch on top
# (abl/lib_ntacc.so), the default bench line, rocprofv3 stats + PMC at C3 and C4
set -o pipefail
mkdir -p gpurun_out/r03zb
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03zb/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zb/smoke.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03zb/ab "c3 c4 c5" $L abl/lib_evdt.so abl/lib_ntacc.so || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03zb/bench.json 2> gpurun_out/r03zb/bench.err || exit 1
bash profiles/run_profiles.sh r03zb_c3 --config c3 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03zb_c4 --config c4 > /dev/null 2>&1 || exit 1
