#!/bin/bash
# round 5 (ad): the slot table with the second admitted candidate in the same line -- the whole
# GPU suite, then the build against r05ac's (profiles/ablib/lib_r05ac.so: slots without it) on
# C5 (table by default) and, with the table forced (IRT_SLOTS=1), C3s and C3
set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ablib/lib_r05ac.so
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c5" $B $L || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $B@IRT_SLOTS=1 $L@IRT_SLOTS=1 $L@IRT_SLOTS=0 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3s" $B@IRT_SLOTS=1 $L@IRT_SLOTS=1 $L@IRT_SLOTS=0 || exit 1
