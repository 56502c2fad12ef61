#!/bin/bash
# round 5 (y): the build with measured-cost work items against the r05q build
# (profiles/ablib/lib_r05q.so) on the chained configs and single C3 frames -- the kernel's
# workgroup mapping grew (SGPR spills 105 -> 117)
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ablib/lib_r05q.so
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $B $L || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $B $L || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s c5 c3t" $B $L || exit 1
