#!/bin/bash
# round 5 (r): measured-cost workgroup order (IRT_SCHED=1: longest 64x64 tiles first, from the
# durations every 8th launch records) on single-frame launches of C3t, whose limb packets run
# 190-240 us against a 29 us median, and of C3 -- interleaved A/B
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=1 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab1 "c3t c3" $L $L@IRT_SCHED=1 || exit 1
IRT_SCHED=1 timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 --warmup 20 > $O/wg_c3t_b1_sched.jsonl 2> $O/wg_c3t_b1_sched.err || exit 1
