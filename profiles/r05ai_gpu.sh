#!/bin/bash
# round 5 (ai): the slot kernel's slot and block loads with the non-temporal hint (profiles/ablib/
# lib_r05ai.so) against the final tree (lib_r05ah.so) on C5, and C3s with the table forced
set -o pipefail
O=gpurun_out/r05ai
mkdir -p $O
L=profiles/ablib/lib_r05ai.so
B=profiles/ablib/lib_r05ah.so
BATCH=8 ROUNDS=3 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab8 "c5" $B $L || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3s" $B@IRT_SLOTS=1 $L@IRT_SLOTS=1 || exit 1
