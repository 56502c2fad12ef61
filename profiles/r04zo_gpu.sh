# round 4 (zo): -amdgpu-schedule-metric-bias=100 (x3) against the default, three interleaved
# rounds at C3, C4 and C5 (r04zl had it within noise at two rounds)
set -o pipefail
O=gpurun_out/r04zo
mkdir -p $O
D=icon-ray-tracing_amd
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3 c4 c5" $D/libicon_rt_hip.so $D/libicon_rt_hip_x3.so || exit 1
