#!/bin/bash
# round 6 (o): two chained frames per wave (OPT_FPAIR = bit 1: 73667873 flat, 73405729 holes):
# the chain tests with it forced and every A/B variant against the default, then the A/B at 8
# chained frames per launch on C3 and C3t (and C3s)
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
A=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip_all.so
IRT_LIB_PATH=$A IRT_RENDER_VARIANT=73405729 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_chain.py > $O/tests_chain.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/tests_variants.log 2>&1 || exit 1
A=icon-ray-tracing_amd/libicon_rt_hip_all.so
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $A@IRT_RENDER_VARIANT=73667872 $A@IRT_RENDER_VARIANT=73667873 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3t" $A@IRT_RENDER_VARIANT=73405728 $A@IRT_RENDER_VARIANT=73405729 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3s" $A@IRT_RENDER_VARIANT=73667872 $A@IRT_RENDER_VARIANT=73667873 || exit 1
