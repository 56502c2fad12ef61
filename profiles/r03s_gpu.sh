# round 3 (s): branch-free atanf reduction (bit-exact), LDS-staged cell headers (OPT_HDRLDS,
# the VERDICT's "LDS-staged column cells" probe), less LDS per workgroup (OPT_LEAN) at 4 and 5
# waves/SIMD; C4 frame mode per rank with measured-cost workgroup order (IRT_SCHED)
set -o pipefail
mkdir -p gpurun_out/r03s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s/gpu_tests.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03s/ab "c3 c3s c5" $L $L@IRT_RENDER_VARIANT=1053696 $L@IRT_RENDER_VARIANT=2102272 $L@IRT_RENDER_VARIANT=2102528 || exit 1
timeout -k 10 400 python3 profiles/rank_step.py --config c4 --modes frame --deals dealt --ranks 1,8 > gpurun_out/r03s/rank_c4_frame.jsonl 2> gpurun_out/r03s/rank_c4_frame.err || exit 1
IRT_SCHED=1 timeout -k 10 400 python3 profiles/rank_step.py --config c4 --modes frame --deals dealt --ranks 1,8 > gpurun_out/r03s/rank_c4_frame_sched1.jsonl 2> gpurun_out/r03s/rank_c4_frame_sched1.err || exit 1
