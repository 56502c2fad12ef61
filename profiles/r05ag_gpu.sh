#!/bin/bash
# round 5 (ag): 64-B slots (two sub-cells of a bin per line; the radial range from the table bin's
# nominal pair) against r05ac's 128-B slots (profiles/ablib/lib_r05ac.so): the slot, locator and
# C5 tests, then C5 (table by default) and, with the table forced, C3s and C3
set -o pipefail
O=gpurun_out/r05ag
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_slots.py tests/test_gpu_parity.py tests/test_gpu_scale.py -k "slot or locator or c5" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
L=profiles/ablib/lib_r05ag.so
B=profiles/ablib/lib_r05ac.so
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c5" $B $L || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $B@IRT_SLOTS=1 $L@IRT_SLOTS=1 $L@IRT_SLOTS=0 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3s" $B@IRT_SLOTS=1 $L@IRT_SLOTS=1 $L@IRT_SLOTS=0 || exit 1
