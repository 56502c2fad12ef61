# round 3 (zf): the spill-free 5-wave build on the big scene (C5, IRT_RENDER_VARIANT=5376)
# against the 4-wave build it gets by default; smoke, the default bench line and rocprofv3
# stats + PMC at C3/C4/C5 on the final tree
set -o pipefail
mkdir -p gpurun_out/r03zf
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03zf/ab "c5" $L $L@IRT_RENDER_VARIANT=5376 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zf/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03zf/bench.json 2> gpurun_out/r03zf/bench.err || exit 1
bash profiles/run_profiles.sh r03zf_c3 --config c3 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03zf_c4 --config c4 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03zf_c5 --config c5 > /dev/null 2>&1 || exit 1
