#!/bin/bash
# round 6 (zm): a sparse transfer function (mean Woodcock samples per acceptance >= 8) builds and uses
# the slot table on scenes whose headers fit the last-level cache: the slot tests, then C3s and C3
# against IRT_SLOTS_SPARSE_TF=0 (3 rounds), then C3s's rocprofv3 + PMC passes (its kernel is now the
# slot form k_render<73663904>)
set -o pipefail
O=gpurun_out/r06zm
mkdir -p $O
L=$(pwd)/icon-ray-tracing_amd/libicon_rt_hip.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_slots.py > $O/tests_slots.log 2>&1 || exit 1
BATCH=8 ROUNDS=3 timeout -k 10 700 bash profiles/ab_multi.sh $O/ab8 "c3s c3" $L "$L@IRT_SLOTS_SPARSE_TF=0" || exit 1
timeout -k 10 700 bash profiles/run_profiles.sh r06zm_c3s --config c3s > $O/prof_c3s.log 2>&1 || exit 1
