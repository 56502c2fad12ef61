#!/bin/bash
# round 6 (y): single-frame C3t with the split threshold at 0.5 and 0.35 of the ideal span (default 1.0,
# quarters) and eighths at 0.5; the C5 frame tests and one C5 bench with the default slot unit (quads)
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
P=icon-ray-tracing_amd
L=$(pwd)/$P/libicon_rt_hip.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_scale.py -k "c5" > $O/tests_c5.log 2>&1 || exit 1
BATCH=1 ROUNDS=4 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab1 "c3t" $L "$L@IRT_SPLIT_FACTOR=0.5" "$L@IRT_SPLIT_FACTOR=0.35" "$L@IRT_SPLIT_FACTOR=0.5@IRT_SPLIT_LG=3" || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c5" $L "$L@IRT_SLOT_SUBS=1" || exit 1
