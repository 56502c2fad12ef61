#!/bin/bash
# round 6 (j): is the C3 raygen VALU-bound?  Three SQ PMC passes of the default bench (instruction
# counts by unit and type, VALU busy and lane utilisation, GRBM_GUI_ACTIVE for the busy
# fractions), each its own run; then host-trap PC sampling of the same run (where the VALU
# instructions are)
set -o pipefail
O=$(pwd)/gpurun_out/r06j
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
B=(python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none)
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INST_CYCLES_SALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $O/pmc_a -o run -- "${B[@]}" > $O/bench_a.json 2> $O/bench_a.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 \
  --output-format csv -d $O/pmc_b -o run -- "${B[@]}" > $O/bench_b.json 2> $O/bench_b.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_ANY \
  --output-format csv -d $O/pmc_c -o run -- "${B[@]}" > $O/bench_c.json 2> $O/bench_c.err || exit 1
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 \
  --output-format csv -d $O/pcs -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none > $O/bench_pcs.json 2> $O/bench_pcs.err || exit 1
