# round 3 (v): 5 waves/SIMD as the default raygen (5376; address recompute only at 5+ waves):
# 4 waves past 16 GiB of scene; full GPU suite, smoke, the default bench line, A/B 5376 vs 5120,
# rocprofv3 stats + PMC traffic at C3 and C5
set -o pipefail
mkdir -p gpurun_out/r03v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03v/bench.json 2> gpurun_out/r03v/bench.err || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03v/ab "c3 c4 c5" $L@IRT_RENDER_VARIANT=5376 $L@IRT_RENDER_VARIANT=5120 $L@IRT_RENDER_VARIANT=2102528 || exit 1
bash profiles/run_profiles.sh r03v_c3 --config c3 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03v_c5 --config c5 > /dev/null 2>&1 || exit 1
