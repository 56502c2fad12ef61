#!/bin/bash
# round 6 (m): VALU / SALU per wave of the pieces of a Woodcock round: the A/B library's in-round
# probe exits (IRT_PROBE_EXIT 8..13, irt_render.hip IRT_ROUND_PROBE) and 4, 5 for reference, the
# A/B library's default kernel, C3 at one launch per frame
set -o pipefail
O=$(pwd)/gpurun_out/r06m
mkdir -p $O
R=$(pwd)
A=$R/icon-ray-tracing_amd/libicon_rt_hip_all.so
cd /tmp && export TMPDIR=/tmp
for P in 4 8 9 10 11 12 13 5; do
  IRT_LIB_PATH=$A IRT_PROBE_EXIT=$P timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES \
    --output-format csv -d $O/pmc_p$P -o run -- python3 $R/bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none > $O/bench_p$P.json 2> $O/bench_p$P.err || exit 1
done
