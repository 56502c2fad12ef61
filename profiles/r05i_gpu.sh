#!/bin/bash
# round 5 (i): samples below the lowest bottom of their sub-cell's candidates skip the candidate
# scan (scenes with holes) -- the GPU suite, then the new build against the previous one
# (profiles/ablib/lib_base.so), interleaved, chained and single-frame launches, and a C3t
# single-frame workgroup timeline
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ablib/lib_base.so
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3t c3" $B $L || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3t" $B $L || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 > $O/wg_c3t_b1.jsonl 2> $O/wg_c3t_b1.err || exit 1
