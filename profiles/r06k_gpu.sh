#!/bin/bash
# round 6 (k): VALU / SALU instructions per wave by region of the C3 raygen, one launch per frame:
# the same SQ pass with the measurement-only probe exits (IRT_PROBE_EXIT 3 = after ray generation
# and the box test, 4 = at the first woodcockFunc, 5 = after it, 7 = the whole ray without the
# pixel write; 0 = everything)
set -o pipefail
O=$(pwd)/gpurun_out/r06k
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 0 3 4 5 7; do
  IRT_PROBE_EXIT=$P timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES \
    --output-format csv -d $O/pmc_p$P -o run -- python3 $R/bench.py --batch 1 --steps 20 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none > $O/bench_p$P.json 2> $O/bench_p$P.err || exit 1
done
