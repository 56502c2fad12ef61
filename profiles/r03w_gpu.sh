# round 3 (w): one-wave workgroups (OPT_WAVEWG with OPT_LEAN: 7 KB of LDS per workgroup, a
# finished wave frees its slot at once) at 4 and 5 waves/SIMD; the cooperative loop's initial
# speculation at 5 waves; C4 frame-mode per-rank shares with the 5-wave default
set -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w/gpu_tests.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03w/ab "c3 c4 c3s c5" $L@IRT_RENDER_VARIANT=5376 $L@IRT_RENDER_VARIANT=6296832 $L@IRT_RENDER_VARIANT=6296576 $L@IRT_RENDER_VARIANT=5376@IRT_COOP_MAXLG=1 || exit 1
timeout -k 10 400 python3 profiles/rank_step.py --config c4 --modes frame,progressive --deals dealt --ranks 1,2,4,8 > gpurun_out/r03w/rank_c4.jsonl 2> gpurun_out/r03w/rank_c4.err || exit 1
