#!/bin/bash
# round 5 (m): (1) rays in the box counted at the ray's end (the box test's LDS add waited for
# the prologue's LDS-DMA tables), (2) OPT_LDSLUT: the LUT's alpha channel in LDS (73405824 /
# 73667968) -- the GPU suite on the LDS-LUT variant, then interleaved A/B against the previous
# build (profiles/ablib/lib_base.so). PART=1: suite + C3; PART=2: C3s, C5, C3t
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ablib/lib_base.so
if [ "${PART:-1}" = 1 ]; then
  IRT_RENDER_VARIANT=73405824 timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite_ldslut.log 2>&1 || exit 1
  BATCH=8 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab8 "c3" $B $L $L@IRT_RENDER_VARIANT=73667968 || exit 1
  BATCH=1 ROUNDS=3 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab1 "c3" $B $L $L@IRT_RENDER_VARIANT=73667968 || exit 1
else
  BATCH=8 ROUNDS=2 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab8 "c3s c5" $B $L $L@IRT_RENDER_VARIANT=73667968 || exit 1
  BATCH=8 ROUNDS=2 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab8 "c3t" $B $L $L@IRT_RENDER_VARIANT=73405824 || exit 1
fi
