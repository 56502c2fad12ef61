#!/bin/bash
# round 5 (l): rays in the box counted at the ray's end instead of at the box test (an LDS add
# there waits for the prologue's LDS-DMA tables) -- against the previous build
# (profiles/ablib/lib_base.so), interleaved
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ablib/lib_base.so
BATCH=8 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab8 "c3" $B $L || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $B $L || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c5 c3t" $B $L || exit 1
