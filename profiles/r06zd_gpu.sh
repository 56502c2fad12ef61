#!/bin/bash
# round 6 (zd): a sample close to one quantised coarse key gathers both candidate height/value blocks
# at once instead of the exact keys, then the block (flat-grid kernels): the whole GPU suite, then
# A/B against the previous kernel (old) at C3 (8 frames and one per launch), C3s, C4, C5
set -o pipefail
O=gpurun_out/r06zd
mkdir -p $O
P=icon-ray-tracing_amd
L=$(pwd)/$P/libicon_rt_hip.so
OLD=$(pwd)/$P/libicon_rt_hip_old.so
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3" $OLD $L || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab1 "c3" $OLD $L || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab8 "c3s c4 c5" $OLD $L || exit 1
