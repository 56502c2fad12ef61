# round 4 (zl): AMDGPU scheduler flags on the raygen (same source, 96 VGPRs, 5 waves, no scratch
# for each): x1 -amdgpu-set-wave-priority, x2 -amdgpu-use-amdgpu-trackers,
# x3 -amdgpu-schedule-metric-bias=100; each library's chained frames against the oracle first
set -o pipefail
O=gpurun_out/r04zl
mkdir -p $O
D=icon-ray-tracing_amd
for x in x1 x2 x3; do
  IRT_LIB_PATH=$D/libicon_rt_hip_$x.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_chain.py > $O/parity_$x.log 2>&1 || exit 1
done
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s c5" $D/libicon_rt_hip.so $D/libicon_rt_hip_x1.so \
  $D/libicon_rt_hip_x2.so $D/libicon_rt_hip_x3.so || exit 1
