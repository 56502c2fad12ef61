#!/bin/bash
# round 6 (n): (1) is 8 KB of LDS per one-wave workgroup what cost OPT_CHAINPF / OPT_ACCPF their
# 6 %?  The product kernel with 512 / 1,024 unused bytes of LDS (IRT_LDS_PAD: 7,480 / 7,992 B per
# workgroup) against the product kernel (6,968 B), C3 8 chained frames; (2) C3t single frames:
# the split packets' parts (IRT_SPLIT_LG 2 = 4 parts, the default; 3 = 8) and threshold
# (IRT_SPLIT_FACTOR 1 = the frame's ideal span, the default; 0.7)
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
P=icon-ray-tracing_amd
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $P/libicon_rt_hip.so $P/libicon_rt_hip_pad512.so $P/libicon_rt_hip_pad1024.so || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 500 bash profiles/ab_multi.sh $O/ab1 "c3t" $P/libicon_rt_hip.so $P/libicon_rt_hip.so@IRT_SPLIT_LG=3 $P/libicon_rt_hip.so@IRT_SPLIT_FACTOR=0.7 $P/libicon_rt_hip.so@IRT_SPLIT_LG=3@IRT_SPLIT_FACTOR=0.7 || exit 1
