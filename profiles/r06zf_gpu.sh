#!/bin/bash
# round 6 (zf): where C3t's extra time goes against C3: the statistics variants of the default kernels
# (73438496 = the holes default | OPT_STATS, 73700640 = the flat one | OPT_STATS: Woodcock rounds per
# wave, locate rounds, entry hops, samples by candidate tests) and the shader-clock regions
# (OPT_TIMING: 73930016 holes, 74192160 flat), single frames and 8 chained frames
set -o pipefail
O=gpurun_out/r06zf
mkdir -p $O
export IRT_LIB_PATH=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 200 python3 profiles/probe.py --config c3 --cases "base;variant=73700640;variant=74192160" --rounds 1 > $O/c3.jsonl 2> $O/c3.err || exit 1
timeout -k 10 200 python3 profiles/probe.py --config c3t --cases "base;variant=73438496;variant=73930016" --rounds 1 > $O/c3t.jsonl 2> $O/c3t.err || exit 1
