# round 4 (n): chained frames in the multi-GPU shares and the timelines
# - every rank's share at N = 1, 2, 4, 8 (profiles/rank_step.py, dealt tiles) with 8 chained
#   frames per launch: C3 and C4, progressive and frame mode
# - workgroup timelines of a chained 8-frame launch at C3 and C3s (4 frames)
# - one-wave workgroups (OPT_WAVEWG | OPT_LEAN, 6296832) against the default at batch 8
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
for cfg in c3 c4; do
  timeout -k 10 400 python3 profiles/rank_step.py --config $cfg --batch 8 --deals dealt --steps 20 > $O/rank_${cfg}_b8.jsonl 2> $O/rank_${cfg}.err || exit 1
done
timeout -k 10 200 python3 profiles/wg_trace.py --config c3 --batch 8 --launches 3 > $O/wg_trace_c3_b8.jsonl 2> $O/wg_trace.err || exit 1
timeout -k 10 200 python3 profiles/wg_trace.py --config c3s --batch 4 --launches 2 > $O/wg_trace_c3s_b4.jsonl 2>> $O/wg_trace.err || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s" $L $LA@IRT_RENDER_VARIANT=6296832 || exit 1
