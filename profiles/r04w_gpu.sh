# round 4 (w): the chained regime (8 frames per launch) against A/B knobs measured before on
# single frames: 4 waves/SIMD one-wave workgroups (6296576), the certified fast lat/lon on the
# one-wave build (39851264), the cooperative loop's speculation (IRT_COOP_MAXLG=1, IRT_COOP_RAMP=2);
# two interleaved rounds at C3, C3s, C5
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 360 --timeout-method thread \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/variants.log 2>&1 || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s c5" $L $LA@IRT_RENDER_VARIANT=6296576 $LA@IRT_RENDER_VARIANT=39851264 \
  $L@IRT_COOP_MAXLG=1 $L@IRT_COOP_RAMP=2 || exit 1
