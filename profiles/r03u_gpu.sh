# round 3 (u): the output addresses recomputed at the end of the raygen (no 64-bit pixel index
# or sample-slot pointer held through the rounds): 4-wave 117 VGPRs, the 5-wave build's 6
# remaining spills all in the prologue/epilogue.  GPU suite; A/B at 4 and 5 waves/SIMD vs a3fdcf3.
set -o pipefail
mkdir -p gpurun_out/r03u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u/gpu_tests.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
B=profiles/ab/lib_a3f.so
bash profiles/ab_multi.sh gpurun_out/r03u/ab "c3 c4 c3s c5" $B $L $L@IRT_RENDER_VARIANT=5376 || exit 1
