#!/bin/bash
# round 5 (o): where a wave's time goes, per region (OPT_TIMING shader clocks of the default
# kernel: 73929984 with the miss mode, 74192128 without), at C3, C3s (comb TF) and C3t
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
export IRT_LIB_PATH=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 200 python3 profiles/probe.py --config c3 --cases "base;variant=74192128" --rounds 3 > $O/timing_c3.jsonl 2> $O/timing_c3.err || exit 1
timeout -k 10 200 python3 profiles/probe.py --config c3 --cases "tf=comb;tf=comb,variant=74192128" --rounds 2 > $O/timing_c3s.jsonl 2> $O/timing_c3s.err || exit 1
timeout -k 10 200 python3 profiles/probe.py --config c3t --cases "base;variant=73929984" --rounds 3 > $O/timing_c3t.jsonl 2> $O/timing_c3t.err || exit 1
