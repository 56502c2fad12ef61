#!/bin/bash
# round 6 (zi): C3t with the void walk's cap at 128 and 8 samples per round (default 32), and the first
# round's lane cap at 2 per ray (IRT_COOP_MAXLG=1), 8 chained frames and one per launch, 4 rounds
set -o pipefail
O=gpurun_out/r06zi
mkdir -p $O
P=$(pwd)/icon-ray-tracing_amd
L=$P/libicon_rt_hip.so
BATCH=8 ROUNDS=4 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab8 "c3t" $L $P/libicon_rt_hip_vr128.so $P/libicon_rt_hip_vr8.so "$L@IRT_COOP_MAXLG=1" || exit 1
BATCH=1 ROUNDS=4 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab1 "c3t" $L $P/libicon_rt_hip_vr128.so $P/libicon_rt_hip_vr8.so "$L@IRT_COOP_MAXLG=1" || exit 1
