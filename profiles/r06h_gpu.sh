#!/bin/bash
# round 6 (h): the solo lanes' void walk also in located mode (OPT_VOIDLOC, variant 1147147552 =
# the holes default | 2^30; IRT_VOIDLOC_FIRST=1: only in a call's first round): terrain frames
# against the oracle with it forced (whole C3t frame, strided pixels, 8-way splits, split packets,
# degenerate terrain), then the A/B on C3t, chained 8-frame launches and single frames
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export IRT_LIB_PATH=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip_all.so
IRT_RENDER_VARIANT=1147147552 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_scale.py -k "c3t and (whole or strided or eight)" \
  tests/test_gpu_parity.py::test_terrain_and_degenerate_records_bit_exact tests/test_gpu_split.py::test_split_packets_equal_unscheduled \
  > $O/tests.log 2>&1 || exit 1
IRT_RENDER_VARIANT=1147147552 IRT_VOIDLOC_FIRST=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_scale.py -k "c3t and whole" > $O/tests_first.log 2>&1 || exit 1
unset IRT_LIB_PATH
A=icon-ray-tracing_amd/libicon_rt_hip_all.so
BATCH=8 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab8 "c3t" $A $A@IRT_RENDER_VARIANT=1147147552 $A@IRT_RENDER_VARIANT=1147147552@IRT_VOIDLOC_FIRST=1 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab1 "c3t" $A $A@IRT_RENDER_VARIANT=1147147552 $A@IRT_RENDER_VARIANT=1147147552@IRT_VOIDLOC_FIRST=1 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab8 "c3" $A $A@IRT_PROBE_EXIT=16 $A@IRT_PROBE_EXIT=17 || exit 1
