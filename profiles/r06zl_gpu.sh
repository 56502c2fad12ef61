#!/bin/bash
# round 6 (zl): the slot table forced on the C3 grid (IRT_SLOTS=1: the default unit there is quads,
# 2.0 GB within the scene's 2.4 GB) with the dealt-out slot misses, against none: C3s and C3, 3 rounds;
# then the slot tests (the saturated unmasked count)
set -o pipefail
O=gpurun_out/r06zl
mkdir -p $O
L=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_slots.py > $O/tests_slots.log 2>&1 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab8 "c3s c3" $L "$L@IRT_SLOTS=1" || exit 1
