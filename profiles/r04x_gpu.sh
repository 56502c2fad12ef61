# round 4 (x): the locator's cube-map resolution in the chained regime (IRT_LOCATOR_SCALE 1.4, 2.0
# against 1.0) at C3 and C5 (8 frames / orbit views per launch), and measured-cost workgroup
# order for single-frame launches with one-wave workgroups (IRT_SCHED=1 / 2, --batch 1) at C3, C4;
# two interleaved rounds
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c5" $L $L@IRT_LOCATOR_SCALE=1.4 $L@IRT_LOCATOR_SCALE=2.0 || exit 1
BATCH=1 ROUNDS=2 bash profiles/ab_multi.sh $O/ab_b1 "c3 c4" $L $L@IRT_SCHED=1 $L@IRT_SCHED=2 || exit 1
