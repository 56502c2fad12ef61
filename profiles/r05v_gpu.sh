#!/bin/bash
# round 5 (v): the split defaults (IRT_SPLIT_FACTOR 1.5, quarters, up to 1,024 packets) against a
# lower threshold and no split on C3t single frames, and measured-cost order with splits forced on
# the flat C3 (off there by default)
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=1 ROUNDS=4 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab1 "c3t" $L $L@IRT_SPLIT_FACTOR=1.2 $L@IRT_SPLIT_LG=0 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $L $L@IRT_SCHED=1 || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 --warmup 24 > $O/wg_c3t_b1.jsonl 2> $O/wg_c3t_b1.err || exit 1
