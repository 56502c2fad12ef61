#!/bin/bash
# round 6 (v): the late-round Tracer reads (classify, getValue, spheres) through fresh_args()
# (-DIRT_FRESH_LATE: 62 spilled SGPRs on flat grids, 73 over terrain) against the new default (65 /
# 87) and the committed round-6 kernel ("old", 108 / 120); frames with the late build first
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
P=icon-ray-tracing_amd
export IRT_LIB_PATH=$(pwd)/$P/libicon_rt_hip_late.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_split.py > $O/tests_late_chain.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "(c3 or c3t) and (whole or eight)" > $O/tests_late_scale.log 2>&1 || exit 1
unset IRT_LIB_PATH
BATCH=8 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3 c3t" $P/libicon_rt_hip_old.so $P/libicon_rt_hip.so $P/libicon_rt_hip_late.so || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab1 "c3 c3t" $P/libicon_rt_hip_old.so $P/libicon_rt_hip.so $P/libicon_rt_hip_late.so || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s c5" $P/libicon_rt_hip_old.so $P/libicon_rt_hip.so $P/libicon_rt_hip_late.so || exit 1
