#!/bin/bash
# round 5 (p): A/B variants of the default -- OPT_XPAIR (an XCD's two blocks of a tile share an
# edge: 73405760 / 73667904), OPT_DPPSCAN (the round's prefix by DPP steps for groups of 2, 4,
# 16, 64: 73405728 / 73667872), OPT_ACCPF (a first frame's accum pixel by LDS-DMA at the wave's
# start: 73405712 / 73667856).  PART=1: the GPU suite on the DPP variant, chain/parity tests on
# the accum-prefetch variant, full-size identity checks (probe); PART=2: C3 A/B (8 and 1 frames
# per launch); PART=3: C3s, C5, C3t A/B
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
case "${PART:-1}" in
1)
  IRT_RENDER_VARIANT=73405728 timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite_dppscan.log 2>&1 || exit 1
  IRT_RENDER_VARIANT=73405712 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_accpf.log 2>&1 || exit 1
  timeout -k 10 200 python3 profiles/probe.py --config c3 --cases "tf=comb;tf=comb,variant=73667872;tf=comb,variant=73667904;tf=comb,variant=73667856;base;variant=73667872;variant=73667904;variant=73667856" --rounds 2 > $O/probe_c3.jsonl 2> $O/probe_c3.err || exit 1
  ;;
2)
  BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $L $L@IRT_RENDER_VARIANT=73667904 $L@IRT_RENDER_VARIANT=73667872 $L@IRT_RENDER_VARIANT=73667856 || exit 1
  BATCH=1 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab1 "c3" $L $L@IRT_RENDER_VARIANT=73667904 $L@IRT_RENDER_VARIANT=73667872 $L@IRT_RENDER_VARIANT=73667856 || exit 1
  ;;
3)
  BATCH=8 ROUNDS=2 timeout -k 10 600 bash profiles/ab_multi.sh $O/ab8 "c3s c5" $L $L@IRT_RENDER_VARIANT=73667904 $L@IRT_RENDER_VARIANT=73667872 $L@IRT_RENDER_VARIANT=73667856 || exit 1
  BATCH=8 ROUNDS=2 timeout -k 10 300 bash profiles/ab_multi.sh $O/ab8 "c3t" $L $L@IRT_RENDER_VARIANT=73405760 $L@IRT_RENDER_VARIANT=73405728 $L@IRT_RENDER_VARIANT=73405712 || exit 1
  ;;
esac
