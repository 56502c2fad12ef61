#!/bin/bash
# round 5 (w): measured-cost work items -- packets longer than the frame's ideal span in quarters,
# those over 1.5 x the median whole, all ahead of the regular order -- tests, then single-frame
# A/B on C3t (default, no items, halves) and on C3 with the order forced (off by default there)
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -k "split or sched or variant" -x -v --timeout 120 --timeout-method thread > $O/tests_split.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=1 ROUNDS=4 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab1 "c3t" $L $L@IRT_SPLIT_FACTOR=0 $L@IRT_SPLIT_LG=1 $L@IRT_SPLIT_LG=0 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $L $L@IRT_SCHED=1 || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 --warmup 24 > $O/wg_c3t_b1.jsonl 2> $O/wg_c3t_b1.err || exit 1
