#!/bin/bash
# round 6 (zc): the slot copy = the candidate that is the first admitted one of the most of the unit's
# sub-cells (was: the unit's lowest admitted one): slot tests, then C5 with quads (default) against
# pairs and one sub-cell per slot, 3 rounds
set -o pipefail
O=gpurun_out/r06zc
mkdir -p $O
P=icon-ray-tracing_amd
L=$(pwd)/$P/libicon_rt_hip.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_slots.py \
  "tests/test_gpu_parity.py::test_device_locator_slot_table" > $O/tests_slots.log 2>&1 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab8 "c5" $L "$L@IRT_SLOT_SUBS=2" "$L@IRT_SLOT_SUBS=1" || exit 1
