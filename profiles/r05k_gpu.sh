#!/bin/bash
# round 5 (k): the LCG-jump and logf tables loaded into LDS by LDS-DMA without a prologue wait
# (OPT_DMATAB, 73405696 / 73667840) against the default (6296832 / 6558976): the variant tests,
# then interleaved bench runs, 8 chained frames per launch and one launch per frame
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "variant" > $O/test_variants.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=8 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab8 "c3" $L@IRT_RENDER_VARIANT=6558976 $L@IRT_RENDER_VARIANT=73667840 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $L@IRT_RENDER_VARIANT=6558976 $L@IRT_RENDER_VARIANT=73667840 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3s c5" $L@IRT_RENDER_VARIANT=6558976 $L@IRT_RENDER_VARIANT=73667840 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 200 bash profiles/ab_multi.sh $O/ab8 "c3t" $L@IRT_RENDER_VARIANT=6296832 $L@IRT_RENDER_VARIANT=73405696 || exit 1
