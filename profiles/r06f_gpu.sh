#!/bin/bash
# round 6 (f): a chained frame's accum pixel prefetched by LDS-DMA at the box test (OPT_CHAINPF = 1)
# and the first frame's (OPT_ACCPF = 16, re-measured on round 6's kernels), against the default:
# C3 (flat forms 73667872 / +1 / +16 / +17) at 8 chained frames and at one frame per launch, C3t
# (holes forms 73405728 / +1 / +16 / +17) chained; then the variant-identity test on the A/B library
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
A=icon-ray-tracing_amd/libicon_rt_hip_all.so
BATCH=8 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab8 "c3" $A@IRT_RENDER_VARIANT=73667872 $A@IRT_RENDER_VARIANT=73667873 $A@IRT_RENDER_VARIANT=73667888 $A@IRT_RENDER_VARIANT=73667889 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab1 "c3" $A@IRT_RENDER_VARIANT=73667872 $A@IRT_RENDER_VARIANT=73667888 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab8 "c3t" $A@IRT_RENDER_VARIANT=73405728 $A@IRT_RENDER_VARIANT=73405729 $A@IRT_RENDER_VARIANT=73405745 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/tests.log 2>&1 || exit 1
