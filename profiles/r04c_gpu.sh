# round 4 (c): the persistent launch with per-XCD queues (C3, default and comb TF); interleaved
# A/B of the round-3 kernel (ab/lib_base.so), the default build and the certified fast lat/lon
# (OPT_FASTSPH, 33559808) at C3 and C5; C5's locator resolution (IRT_LOCATOR_SCALE 0.7 / 0.5)
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 300 python3 profiles/probe.py --config c3 --rounds 3 --frames 20 \
  --cases 'base;IRT_QUEUE=1;IRT_QUEUE=1,IRT_QUEUE_WGS=4;tf=comb;tf=comb,IRT_QUEUE=1' \
  > $O/probe_queue_c3.jsonl 2> $O/probe_queue_c3.err || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c5" ab/lib_base.so $L $LA@IRT_RENDER_VARIANT=33559808 || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c5" $L@IRT_LOCATOR_SCALE=0.7 $L@IRT_LOCATOR_SCALE=0.5 || exit 1
