# round 4 (zf): six waves/SIMD one-wave workgroups (6297088: 80 VGPRs, 60 B of scratch) against
# the 5-wave default in the chained regime; variants test first, two interleaved rounds
set -o pipefail
O=gpurun_out/r04zf
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 360 --timeout-method thread \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/variants.log 2>&1 || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s c5" $L $LA@IRT_RENDER_VARIANT=6297088 || exit 1
