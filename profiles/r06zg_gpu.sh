#!/bin/bash
# round 6 (zg): the void walk in located mode (OPT_VOIDLOC, variant 1147147552 = the holes default |
# OPT_VOIDLOC) re-measured on the final tree's kernels: C3t 8 chained frames and one per launch, 4 rounds
set -o pipefail
O=gpurun_out/r06zg
mkdir -p $O
A=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip_all.so
BATCH=8 ROUNDS=4 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3t" $A "$A@IRT_RENDER_VARIANT=1147147552" || exit 1
BATCH=1 ROUNDS=4 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab1 "c3t" $A "$A@IRT_RENDER_VARIANT=1147147552" || exit 1
