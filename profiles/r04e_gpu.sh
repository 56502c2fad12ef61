# round 4 (e): the batched zero-length sdda walk.  GPU suite (bit-exactness, whole frames at
# C2-C5); the strong-scaling (frame mode) rank share at C3 and C4, N = 1 and 8, round-3 kernel
# (ab/lib_base.so) against this build, and this build stopped after ray generation + boxTest
# (IRT_PROBE_EXIT=3), at the first woodcockFunc (4), after it (5); full-frame A/B at C3, C5
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for cfg in c3 c4; do
  IRT_LIB_PATH=ab/lib_base.so timeout -k 10 300 python3 profiles/rank_step.py --config $cfg --ranks 1,8 --modes frame --deals dealt \
    > $O/rank_${cfg}_base.jsonl 2> $O/rank_${cfg}_base.err || exit 1
  for ex in 3 4 5 0; do
    IRT_PROBE_EXIT=$ex timeout -k 10 300 python3 profiles/rank_step.py --config $cfg --ranks 1,8 --modes frame --deals dealt \
      > $O/rank_${cfg}_exit$ex.jsonl 2> $O/rank_${cfg}_exit$ex.err || exit 1
  done
done
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3 c5" ab/lib_base.so icon-ray-tracing_amd/libicon_rt_hip.so || exit 1
