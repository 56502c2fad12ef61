#!/bin/bash
# round 6 (r): is the C3 raygen's time sensitive to VALU work?  The probe build (IRT_PROBE_BUILD)
# with 200 extra v_nop per wave in the ray setup (IRT_PROBE_EXIT=30) or 100 per Woodcock round
# (31) against itself (0): bench A/B at 8 chained frames and one launch per frame, and the SQ
# pass (VALU per wave) of each
set -o pipefail
O=$(pwd)/gpurun_out/r06r
mkdir -p $O
R=$(pwd)
P=icon-ray-tracing_amd/libicon_rt_hip_probe.so
BATCH=8 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab8 "c3" $P $P@IRT_PROBE_EXIT=30 $P@IRT_PROBE_EXIT=31 || exit 1
BATCH=1 ROUNDS=3 timeout -k 10 400 bash profiles/ab_multi.sh $O/ab1 "c3" $P $P@IRT_PROBE_EXIT=30 $P@IRT_PROBE_EXIT=31 || exit 1
cd /tmp && export TMPDIR=/tmp
for X in 0 30 31; do
  IRT_LIB_PATH=$R/$P IRT_PROBE_EXIT=$X timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_x$X -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none > $O/bench_x$X.json 2> $O/bench_x$X.err || exit 1
done
