# round 3 (m): exact double-product division by the per-launch divisors -- parity + A/B
set -o pipefail
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_grid.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03m/gpu_tests.log 2>&1 || exit 1
bash profiles/ab_libs.sh gpurun_out/r03m/ab profiles/ab/libicon_rt_hip_base.so c3 c3s
