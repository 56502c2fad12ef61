# round 4 (i): OPT_PAIR (268440832: the wave-wide scan's first step tests each lane's first
# two candidates, both entries gathered together) -- every A/B variant bit-identical on the
# A/B library, then interleaved against the default at C3s, C3, C5
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 360 --timeout-method thread \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/variants.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3s c3 c5" $L $LA@IRT_RENDER_VARIANT=268440832 || exit 1
