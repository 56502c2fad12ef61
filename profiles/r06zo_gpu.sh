#!/bin/bash
# round 6 (zo): slot units of 16 sub-cells (one slot per cell and bin; masks now in words 20-23): the slot
# tests and the slot locator, then C3s (sparse TF: quads by default) and C5 (quads) against the same
# with IRT_SLOT_SUBS=16 and against the previous library (old, masks in word 18), 3 rounds
set -o pipefail
O=gpurun_out/r06zo
mkdir -p $O
P=$(pwd)/icon-ray-tracing_amd
L=$P/libicon_rt_hip.so
OLD=$P/libicon_rt_hip_old.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_slots.py \
  "tests/test_gpu_parity.py::test_device_locator_slot_table" > $O/tests_slots.log 2>&1 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab8 "c3s c5" $OLD $L "$L@IRT_SLOT_SUBS=16" || exit 1
