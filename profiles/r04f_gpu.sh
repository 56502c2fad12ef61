# round 4 (f): first the GPU suite on this tree (done markers recorded every 8th launch,
# irt_set_statistics); the header touch at the ray's entry (OPT_HDRPF, 67114240) against the
# default at C3, C3s, C5 (interleaved); the strong-scaling rank share at C3: an empty launch
# (IRT_PROBE_EXIT=1), without and with statistics, and the kernel durations under rocprofv3
# (are the N = 8 steps GPU- or host-bound?); the persistent launch without the fetch prefetch
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
ROOT=$(pwd)
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python3 profiles/probe.py --config c3 --rounds 3 --frames 20 --cases 'base;IRT_QUEUE=1;IRT_QUEUE=1,IRT_QUEUE_WGS=2;IRT_COUNTERS=off' \
  > $O/probe_queue_c3.jsonl 2> $O/probe_queue_c3.err || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c3s c5" $L $LA@IRT_RENDER_VARIANT=67114240 || exit 1
for envs in "IRT_PROBE_EXIT=1" "IRT_COUNTERS=off" "IRT_COUNTERS=on"; do
  n=${envs//=/_}
  env $envs timeout -k 10 300 python3 profiles/rank_step.py --config c3 --ranks 1,8 --modes frame --deals dealt \
    > $O/rank_c3_$n.jsonl 2> $O/rank_c3_$n.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/rank_prof -o run \
  -- python3 $ROOT/profiles/rank_step.py --config c3 --ranks 8 --modes frame --deals dealt --steps 50 \
  > $ROOT/$O/rank_c3_prof.jsonl 2> $ROOT/$O/rank_c3_prof.err || exit 1
