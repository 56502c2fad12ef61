#!/bin/bash
# round 5 (ab): rocprofv3 kernel trace + FETCH/WRITE/L2 passes with and without the slot table
# (IRT_SLOTS) on C3 (slower with it) and C5 (faster with it)
set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
IRT_SLOTS=1 timeout -k 10 600 bash profiles/run_profiles.sh r05ab_c3_slots --config c3 > $O/prof_c3_slots.log 2>&1 || exit 1
IRT_SLOTS=0 timeout -k 10 600 bash profiles/run_profiles.sh r05ab_c3_noslots --config c3 > $O/prof_c3_noslots.log 2>&1 || exit 1
IRT_SLOTS=1 timeout -k 10 600 bash profiles/run_profiles.sh r05ab_c5_slots --config c5 > $O/prof_c5_slots.log 2>&1 || exit 1
IRT_SLOTS=1 timeout -k 10 600 bash profiles/run_profiles.sh r05ab_c3s_slots --config c3s > $O/prof_c3s_slots.log 2>&1 || exit 1
