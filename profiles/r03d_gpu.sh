# round 3 (d): 64-B candidate entries -- full GPU suite, A/B vs the round-2 layout, PMC traffic
set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/gpu_tests.log 2>&1 || exit 1
bash profiles/ab_libs.sh gpurun_out/r03d/ab profiles/ab/libicon_rt_hip_base.so c3 c5 c3s c4 || exit 1
bash profiles/run_profiles.sh r03d_c3 --config c3 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r03d_c5 --config c5 > /dev/null 2>&1 || exit 1
