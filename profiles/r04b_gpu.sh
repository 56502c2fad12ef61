# round 4 (b): interleaved A/B on one box (profiles/ab_multi.sh, bench.py kernel ms): the
# round-3 kernel (ab/lib_base.so) against the certified fast lat/lon, and the persistent
# launch (IRT_QUEUE=1), at C3, C3s and C5
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s c5" ab/lib_base.so $L $L@IRT_QUEUE=1 || exit 1
