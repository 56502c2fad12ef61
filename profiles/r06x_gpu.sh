#!/bin/bash
# round 6 (x): slot units of 4 / 2 / 1 sub-cells where a lane whose sub-cell does not admit the unit's
# first candidate deals all of its own candidates out (no gather of its own on the chain), against
# no table; C5 and C3s (table forced), after the slot tests
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
P=icon-ray-tracing_amd
L=$(pwd)/$P/libicon_rt_hip.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_slots.py \
  "tests/test_gpu_parity.py::test_device_locator_slot_table" > $O/tests_slots.log 2>&1 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab8 "c5" "$L@IRT_SLOT_SUBS=4" "$L@IRT_SLOT_SUBS=2" "$L@IRT_SLOT_SUBS=1" "$L@IRT_SLOTS=0" || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s" "$L@IRT_SLOTS=1@IRT_SLOT_SUBS=2" "$L@IRT_SLOTS=1@IRT_SLOT_SUBS=1" "$L@IRT_SLOTS=0" || exit 1
