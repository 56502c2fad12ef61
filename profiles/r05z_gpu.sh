#!/bin/bash
# round 5 (z): the split logic in its own instantiation of the default kernels (OPT_SPLIT, used only
# by single frames with measured-cost work items) -- the whole GPU suite, then the build against
# r05q (profiles/ablib/lib_r05q.so) on chained C3/C3s/C5/C3t and single C3, and single C3t frames
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ablib/lib_r05q.so
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $B $L || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3 c3t" $B $L || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s c5 c3t" $B $L || exit 1
