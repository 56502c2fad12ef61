#!/bin/bash
# round 5 (t): the split threshold (IRT_SPLIT_FACTOR 4 / 3 / 2, halves and quarters) on C3t
# single frames -- interleaved A/B and workgroup timelines naming the longest workgroups
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=1 ROUNDS=3 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab1 "c3t" $L $L@IRT_SPLIT_FACTOR=3 $L@IRT_SPLIT_FACTOR=2 $L@IRT_SPLIT_FACTOR=2@IRT_SPLIT_LG=2 $L@IRT_SPLIT_FACTOR=3@IRT_SPLIT_LG=2 || exit 1
for f in 4 2; do
  IRT_SPLIT_FACTOR=$f timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 --warmup 24 > $O/wg_c3t_b1_f$f.jsonl 2> $O/wg_c3t_b1_f$f.err || exit 1
done
