#!/bin/bash
# round 5 (h): a single frame's tail in half packets (IRT_SPLIT_TAIL) -- bit-exactness tests,
# workgroup timelines of single C3 frames split and unsplit, and single-frame launches
# (BATCH=1) A/B over the split size, interleaved
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_split.py > $O/test_split.log 2>&1 || exit 1
for s in 0 2560 5120; do
  IRT_SPLIT_TAIL=$s timeout -k 10 180 python3 profiles/wg_trace.py --config c3 --launches 2 > $O/wg_c3_b1_s$s.jsonl 2> $O/wg_c3_b1_s$s.err || exit 1
done
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=1 ROUNDS=3 timeout -k 10 840 bash profiles/ab_multi.sh $O/ab "c3 c4" $L@IRT_SPLIT_TAIL=0 $L@IRT_SPLIT_TAIL=1280 \
  $L@IRT_SPLIT_TAIL=2560 $L@IRT_SPLIT_TAIL=5120 $L@IRT_SPLIT_TAIL=8192 || exit 1
