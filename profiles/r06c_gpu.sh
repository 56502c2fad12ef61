#!/bin/bash
# round 6 (c): the quad-bound miss test (header words 24..31; Tracer::locate_wave kHoleSkip):
# correctness (device build == host build, locators, whole C3t frames, splits, chains) and the
# A/B on C3t: default 73405728 (with the test) against 73405732 (OPT_NOHOLESKIP), chained
# 8-frame launches and single frames, interleaved on one box
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_build.py \
  "tests/test_gpu_parity.py::test_device_locator_matches_host_restatement" tests/test_gpu_split.py tests/test_gpu_chain.py \
  "tests/test_gpu_scale.py" -k "not c5" > $O/tests.log 2>&1 || exit 1
A=icon-ray-tracing_amd/libicon_rt_hip_all.so
BATCH=8 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3t" $A $A@IRT_RENDER_VARIANT=73405732 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab1 "c3t" $A $A@IRT_RENDER_VARIANT=73405732 || exit 1
