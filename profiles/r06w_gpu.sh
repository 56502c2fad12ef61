#!/bin/bash
# round 6 (w): the slot table by units of 2 x 2 sub-cells (quads, IRT_SLOT_SUBS=4, the new default:
# a quarter of the table) against pairs (2) and round 5's one sub-cell per slot (1), and no table
# (IRT_SLOTS=0); the GPU slot tests first
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
P=icon-ray-tracing_amd
L=$(pwd)/$P/libicon_rt_hip.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_slots.py \
  "tests/test_gpu_parity.py::test_device_locator_slot_table" > $O/tests_slots.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_scale.py -k "c5" > $O/tests_c5.log 2>&1 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab8 "c5" $L "$L@IRT_SLOT_SUBS=2" "$L@IRT_SLOT_SUBS=1" "$L@IRT_SLOTS=0" || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s" "$L@IRT_SLOTS=1" "$L@IRT_SLOTS=1@IRT_SLOT_SUBS=1" $L || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" "$L@IRT_SLOTS=1" $L || exit 1
