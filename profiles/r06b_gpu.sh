#!/bin/bash
# round 6 (b): where a wave's time goes by region (OPT_TIMING shader clocks; 74192160 = the flat
# default 73667872 | OPT_TIMING, 73930016 = the holes default 73405728 | OPT_TIMING), single
# frames at C3 and C3t, to pick the round's kernel work
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
export IRT_LIB_PATH=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 200 python3 profiles/probe.py --config c3 --cases "base;variant=74192160" --rounds 2 > $O/timing_c3.jsonl 2> $O/timing_c3.err || exit 1
timeout -k 10 200 python3 profiles/probe.py --config c3t --cases "base;variant=73930016" --rounds 2 > $O/timing_c3t.jsonl 2> $O/timing_c3t.err || exit 1
timeout -k 10 200 python3 profiles/probe.py --config c3 --cases "tf=comb;tf=comb,variant=74192160" --rounds 1 > $O/timing_c3s.jsonl 2> $O/timing_c3s.err || exit 1
