# round 4 (zc): 2 x 2 sub-cells per cube-map cell (IRT_SUBCELLS=2: 64-B cell headers, coarser
# candidate masks; profiles/ablib/lib_sub2.so) -- its device build and frames against the host
# restatement and the oracle, then three interleaved rounds against the shipped build at C3,
# C3s, C4, C5 (8 frames / views per launch)
set -o pipefail
O=gpurun_out/r04zc
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
S=profiles/ablib/lib_sub2.so
IRT_LIB_PATH=$S timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_build.py \
  tests/test_gpu_chain.py "tests/test_gpu_parity.py::test_frame_bit_exact" \
  "tests/test_gpu_parity.py::test_gpu_matches_reference_golden" > $O/tests_sub2.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3 c3s c4 c5" $L $S || exit 1
