# round 4 (o): chained frames in lagged groups (IRT_CHAIN_LAG: block b's frames D workgroups apart,
# for L2 reuse across frames) and one-wave workgroups (6296832; its prewarm launched 256 threads
# before the fix) against the default, 8 frames per launch; the variants and chain tests first
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_chain.py \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/tests.log 2>&1 || exit 1
IRT_CHAIN_LAG=256 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py > $O/tests_lag.log 2>&1 || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s" $L $L@IRT_CHAIN_LAG=256 $L@IRT_CHAIN_LAG=640 $L@IRT_CHAIN_LAG=1280 $LA@IRT_RENDER_VARIANT=6296832 || exit 1
