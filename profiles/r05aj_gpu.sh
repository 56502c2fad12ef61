#!/bin/bash
# round 5 (aj): the cooperative loop's lane caps re-measured on the round-5 kernels (tuned in
# round 2): first-round cap 2^IRT_COOP_MAXLG (default 0), IRT_COOP_RAMP doublings per round
# (default 1) -- every setting renders the same frame
set -o pipefail
O=gpurun_out/r05aj
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=8 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3" $L $L@IRT_COOP_RAMP=2 $L@IRT_COOP_MAXLG=1 $L@IRT_COOP_MAXLG=1@IRT_COOP_RAMP=2 $L@IRT_COOP_RAMP=3 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s c3t" $L $L@IRT_COOP_RAMP=2 $L@IRT_COOP_MAXLG=1 || exit 1
