# round 3 (zg): 5 vs 4 waves on the big scene after the spill removal, six interleaved rounds
# (C5, IRT_RENDER_VARIANT=5376 vs the default 4-wave choice past 16 GiB), and C3s once more
set -o pipefail
mkdir -p gpurun_out/r03zg
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03zg/ab "c5" $L $L@IRT_RENDER_VARIANT=5376 || exit 1
bash profiles/ab_multi.sh gpurun_out/r03zg/ab "c5" $L $L@IRT_RENDER_VARIANT=5376 || exit 1
bash profiles/ab_multi.sh gpurun_out/r03zg/ab "c3s" $L abl/lib_prespill.so || exit 1
