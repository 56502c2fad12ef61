# round 3 (y): the statistics epilogue before the pixel stores (render_pixel_coop's `finish`):
# full GPU suite + smoke on the new kernel, A/B against the previous HEAD build (abl/lib_head.so),
# the default bench line, rocprofv3 stats + PMC at C3
set -o pipefail
mkdir -p gpurun_out/r03y
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03y/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y/smoke.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03y/ab "c3 c4 c3s" $L abl/lib_head.so || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03y/bench.json 2> gpurun_out/r03y/bench.err || exit 1
bash profiles/run_profiles.sh r03y_c3 --config c3 > /dev/null 2>&1 || exit 1
