# round 4 (y): two-wave workgroups (OPT_WAVEWG2 | OPT_LEAN, 538973440: a block's packets in
# pairs sharing a CU's L1) against the one-wave default; variants + chain tests first, then
# three interleaved rounds at C3, C3s, C4, C5 (8 frames / views per launch)
set -o pipefail
O=gpurun_out/r04y
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_chain.py \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/tests.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3 c3s c4 c5" $L $LA@IRT_RENDER_VARIANT=538973440 || exit 1
