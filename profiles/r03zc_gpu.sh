# round 3 (zc): streaming pixel stores + accum prefetch in the 5-wave builds only (the 4-wave
# build for scenes over 16 GiB keeps plain ones): full GPU suite + smoke, A/B against the
# previous default (abl/lib_evdt.so), the default bench line, rocprofv3 stats + PMC at C3/C4/C5
set -o pipefail
mkdir -p gpurun_out/r03zc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03zc/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zc/smoke.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03zc/ab "c3 c4 c5 c3s" $L abl/lib_evdt.so || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03zc/bench.json 2> gpurun_out/r03zc/bench.err || exit 1
bash profiles/run_profiles.sh r03zc_c3 --config c3 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03zc_c4 --config c4 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03zc_c5 --config c5 > /dev/null 2>&1 || exit 1
