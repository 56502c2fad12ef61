#!/bin/bash
# round 5 (u): the split threshold around IRT_SPLIT_FACTOR 2 with quarters on C3t single frames
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=1 ROUNDS=4 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab1 "c3t" $L@IRT_SPLIT_FACTOR=2@IRT_SPLIT_LG=2 $L@IRT_SPLIT_FACTOR=1.5@IRT_SPLIT_LG=2 $L@IRT_SPLIT_FACTOR=2@IRT_SPLIT_LG=1 $L@IRT_SPLIT_FACTOR=1.5@IRT_SPLIT_LG=3 $L@IRT_SPLIT_LG=0 || exit 1
IRT_SPLIT_FACTOR=2 IRT_SPLIT_LG=2 timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 --warmup 24 > $O/wg_c3t_b1_f2lg2.jsonl 2> $O/wg_c3t_b1_f2lg2.err || exit 1
