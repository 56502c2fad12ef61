#!/bin/bash
# round 6 (d): C3t A/B of the miss-mode kernel's two void measures: default 73405728 (the quad-bound
# test + the solo lanes' void walk), 73405730 (test only, OPT_NOVOIDRUN), 73405732 (neither,
# OPT_NOHOLESKIP); chained 8-frame launches and single frames; then the frame tests on C3t
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
A=icon-ray-tracing_amd/libicon_rt_hip_all.so
BATCH=8 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3t" $A $A@IRT_RENDER_VARIANT=73405730 $A@IRT_RENDER_VARIANT=73405732 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab1 "c3t" $A $A@IRT_RENDER_VARIANT=73405730 $A@IRT_RENDER_VARIANT=73405732 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_device_locator_matches_host_restatement" tests/test_gpu_split.py tests/test_gpu_chain.py \
  tests/test_gpu_scale.py -k "not c5" > $O/tests.log 2>&1 || exit 1
