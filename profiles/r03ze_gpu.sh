# round 3 (ze): no scratch spills in the 5-wave kernel (the thread index, the pixel's in-block
# coordinates and the s_entry slot recomputed from an SGPR wave base + the lane id after/inside
# the rounds instead of 24 B per lane held in scratch; the block index kept scalar): GPU suite
# on it, A/B against the previous build (abl/lib_cur.so); then the streaming stores of the
# progressive batch's samples (abl/lib_ntsamp.so vs abl/lib_cur.so) with profiles/rank_step.py
set -o pipefail
mkdir -p gpurun_out/r03ze
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ze/gpu_tests.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03ze/ab "c3 c4 c5 c3s" $L abl/lib_cur.so || exit 1
for round in 1 2; do
  for lib in abl/lib_cur.so abl/lib_ntsamp.so; do
    n=$(basename $lib .so)
    IRT_LIB_PATH=$lib timeout -k 10 300 python3 profiles/rank_step.py --config c3 --ranks 2,8 \
      --modes progressive --deals dealt --steps 40 >> gpurun_out/r03ze/rs_${n}_c3.jsonl 2>> gpurun_out/r03ze/rs_${n}_c3.err || exit 1
  done
done
