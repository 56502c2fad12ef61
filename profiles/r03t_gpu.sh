# round 3 (t): uniform-derived values recomputed at their uses instead of held in VGPRs
# (opaque_u: the cube-map scale, (float)(dims-1), (float)lutSize, sceneEPS; wrap_coord without
# the hoisted division reciprocals): 4-wave kernel 127 -> 118 VGPRs, the 5-wave build's spills
# 18 -> 9 and none left inside the loops; OPT_DEALALL (every candidate dealt out, one entry
# gather per round).  GPU suite; A/B vs e41ea77 at 4 and 5 waves/SIMD.
set -o pipefail
mkdir -p gpurun_out/r03t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03t/gpu_tests.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ab/lib_e41.so
bash profiles/ab_multi.sh gpurun_out/r03t/ab "c3 c3s c5" $B $L $L@IRT_RENDER_VARIANT=5376 $L@IRT_RENDER_VARIANT=8393728 $L@IRT_RENDER_VARIANT=8393984 || exit 1
