#!/bin/bash
# round 5 (s): measured-cost scheduling with split packets (the costliest packets of a single
# frame rendered in 2 or 4 parts first) -- its tests, then C3t/C3 single frames A/B (split in
# halves by default, quarters, no split) and C3t workgroup timelines
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -k "split or sched or variant" -x -v --timeout 120 --timeout-method thread > $O/tests_split.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=1 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab1 "c3t" $L $L@IRT_SPLIT_LG=2 $L@IRT_SPLIT_LG=0 $L@IRT_SPLIT_FACTOR=2.5 || exit 1
BATCH=1 ROUNDS=2 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $L $L@IRT_SCHED=1 || exit 1
for lg in 1 2; do
  IRT_SPLIT_LG=$lg timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 --warmup 24 > $O/wg_c3t_b1_lg$lg.jsonl 2> $O/wg_c3t_b1_lg$lg.err || exit 1
done
