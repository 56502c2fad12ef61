#!/bin/bash
# round 5 (aa): the slot table (OPT_SLOT: per (cell, sub-cell, bin) the first admitted candidate and
# the list's position in one 128-B line) -- its GPU tests, the whole GPU suite (which runs every
# flat scene through it), then IRT_SLOTS=0 against the table on chained C3/C3s/C4/C5 and single C3
set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_slots.py -x -v --timeout 120 --timeout-method thread > $O/slots_tests.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $L@IRT_SLOTS=0 $L@IRT_SLOTS=1 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $L@IRT_SLOTS=0 $L@IRT_SLOTS=1 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab8 "c3s c4 c5" $L@IRT_SLOTS=0 $L@IRT_SLOTS=1 || exit 1
