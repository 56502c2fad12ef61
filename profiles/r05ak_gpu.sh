#!/bin/bash
# round 5 (ak): the cube-map resolution re-measured at C5 now that it runs with the slot table
# (the table grows with G^2: 83 GB at 0.8 x, 129 GB at 1 x, 171 GB at 1.15 x); C3s with the table
# forced for comparison
set -o pipefail
O=gpurun_out/r05ak
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
BATCH=8 ROUNDS=2 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab8 "c5" $L $L@IRT_LOCATOR_SCALE=0.8 $L@IRT_LOCATOR_SCALE=1.15 || exit 1
