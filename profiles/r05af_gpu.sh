#!/bin/bash
# round 5 (af): address-translation (UTCL1) counters of the raygen with and without the slot table
# at C5 (168 GB resident with it, 39 GB without) and at C3
set -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/r05af
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CNT="TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCR_TCP_STALL_CYCLES_sum"
for spec in c5:1 c5:0 c3:0; do
  cfg=${spec%%:*}; sl=${spec##*:}
  IRT_SLOTS=$sl timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d $O/${cfg}_slots$sl -o run \
    -- python3 $ROOT/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-single-compare > $O/${cfg}_slots$sl.json 2> $O/${cfg}_slots$sl.err || exit 1
done
