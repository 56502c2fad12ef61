# round 4 (p): one-wave workgroups (OPT_WAVEWG | OPT_LEAN at 5 waves/SIMD, 6296832) against the
# default at C3, C3s, C4 (8 chained frames per launch), C5 (orbit: one frame per launch) and C3
# at one frame per launch; three interleaved rounds on one box
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3 c3s c4 c5" $L $LA@IRT_RENDER_VARIANT=6296832 || exit 1
BATCH=1 ROUNDS=3 bash profiles/ab_multi.sh $O/ab_b1 "c3" $L $LA@IRT_RENDER_VARIANT=6296832 || exit 1
