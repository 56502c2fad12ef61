#!/bin/bash
# round 6 (i): the counters this box offers (rocprofv3 -L), and where a C3 wave waits: one SQ pass
# (wave cycles, any wait, instruction-fetch wait, active cycles by unit) of the default bench
set -o pipefail
O=$(pwd)/gpurun_out/r06i
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2> $O/avail.err || true
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVES \
  --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none > $O/bench_sq.json 2> $O/bench_sq.err || exit 1
