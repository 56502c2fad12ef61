#!/bin/bash
# round 6 (s): VERDICT r05 5b, the SGPR spills.  The ray's state machine reading RenderArgs
# through fresh_args() (-DIRT_FRESH_ARGS: 78 spilled SGPRs on flat grids, 92 over terrain, against
# 102 / 112 of the same source without it and 108 / 120 of the committed kernel, "old"): frames
# against the oracle with the fresh build, then the A/B of the three libraries, interleaved
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
P=icon-ray-tracing_amd
IRT_LIB_PATH=$(pwd)/$P/libicon_rt_hip_fresh.so timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_scale.py -k "(c3 or c3t) and (whole or eight)" tests/test_gpu_chain.py tests/test_gpu_split.py \
  tests/test_gpu_parity.py::test_convert_icon_terrain_bit_exact_with_and_without_miss_mode > $O/tests_fresh.log 2>&1 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3 c3t" $P/libicon_rt_hip_old.so $P/libicon_rt_hip.so $P/libicon_rt_hip_fresh.so || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab1 "c3" $P/libicon_rt_hip_old.so $P/libicon_rt_hip.so $P/libicon_rt_hip_fresh.so || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s c5" $P/libicon_rt_hip_old.so $P/libicon_rt_hip.so $P/libicon_rt_hip_fresh.so || exit 1
