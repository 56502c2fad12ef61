#!/bin/bash
# profiles/pmc_multi.sh OUTDIR VARIANTS [ab_variants args]: the standard counter passes
# (SQ timing, SQ instruction mix, memory hierarchy, HBM fetch/write) over
# profiles/ab_variants.py, one rocprofv3 --pmc pass each (kernel-trace only besides the
# counters; never combined with runtime/sys traces).
set -euo pipefail
OUT=$1; shift
VARS=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
P=profiles/pmc_pass.sh
bash $P $OUT/sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --variants $VARS --rounds 1 --frames 3 --no-check "$@"
bash $P $OUT/sq2 "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH" --variants $VARS --rounds 1 --frames 3 --no-check "$@"
bash $P $OUT/mem "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum" --variants $VARS --rounds 1 --frames 3 --no-check "$@"
bash $P $OUT/tlb "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_REQUEST_sum" --variants $VARS --rounds 1 --frames 3 --no-check "$@"
bash $P $OUT/fetch "FETCH_SIZE" --variants $VARS --rounds 1 --frames 3 --no-check "$@"
