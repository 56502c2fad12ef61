#!/bin/bash
# round 6 (z): the split threshold of scenes with holes at its new default 0.35 against 1.0 (round 5's),
# 0.5, 0.25 and 0.2, single C3t frames, 5 rounds; the split and terrain frame tests first
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
P=icon-ray-tracing_amd
L=$(pwd)/$P/libicon_rt_hip.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_split.py > $O/tests_split.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "c3t" > $O/tests_c3t.log 2>&1 || exit 1
BATCH=1 ROUNDS=5 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab1 "c3t" $L "$L@IRT_SPLIT_FACTOR=1.0" "$L@IRT_SPLIT_FACTOR=0.5" "$L@IRT_SPLIT_FACTOR=0.25" "$L@IRT_SPLIT_FACTOR=0.2" || exit 1
