#!/bin/bash
# round 6 (l): does fewer VALU make C3 faster?  The certified fast lat/lon for the sdda entry/exit
# cells (OPT_FASTSPH on round 6's default: 107222304 flat, 106960160 holes) against the default:
# VALU/SALU per wave (SQ pass, one launch per frame) and the bench A/B (8 chained frames, single
# frames; C3 and C3t)
set -o pipefail
O=$(pwd)/gpurun_out/r06l
mkdir -p $O
R=$(pwd)
A=$R/icon-ray-tracing_amd/libicon_rt_hip_all.so
(cd /tmp && export TMPDIR=/tmp && IRT_LIB_PATH=$A IRT_RENDER_VARIANT=107222304 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES \
    --output-format csv -d $O/pmc_fastsph -o run -- python3 $R/bench.py --batch 1 --steps 20 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none > $O/bench_pmc.json 2> $O/bench_pmc.err) || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $A@IRT_RENDER_VARIANT=73667872 $A@IRT_RENDER_VARIANT=107222304 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab1 "c3" $A@IRT_RENDER_VARIANT=73667872 $A@IRT_RENDER_VARIANT=107222304 || exit 1
BATCH=8 ROUNDS=2 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3t" $A@IRT_RENDER_VARIANT=73405728 $A@IRT_RENDER_VARIANT=106960160 || exit 1
