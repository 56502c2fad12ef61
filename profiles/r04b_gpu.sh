# round 4 (b): interleaved A/B on one box (profiles/ab_multi.sh, bench.py kernel ms): the
# round-3 kernel (ab/lib_base.so) against the certified fast lat/lon at C3, C3s and C5; the
# persistent launch's workgroup count (occupancy query vs IRT_QUEUE_WGS per CU) at C3
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
timeout -k 10 300 python3 profiles/probe.py --config c3 --rounds 3 --frames 20 \
  --cases 'base;IRT_QUEUE=1;IRT_QUEUE=1,IRT_QUEUE_WGS=5;IRT_QUEUE=1,IRT_QUEUE_WGS=4;IRT_QUEUE=1,IRT_QUEUE_WGS=8;IRT_QUEUE=1,IRT_QUEUE_WGS=2' \
  > $O/probe_queue_c3.jsonl 2> $O/probe_queue_c3.err || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s c5" ab/lib_base.so $L || exit 1
