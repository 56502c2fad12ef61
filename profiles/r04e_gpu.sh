# round 4 (e): where the strong-scaling (frame mode, N = 8) rank share's time goes at C3 and
# C4: the same share stopped after ray generation + boxTest (IRT_PROBE_EXIT=3), at the first
# woodcockFunc (4), after it (5), and whole
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
for cfg in c3 c4; do
  for ex in 3 4 5 0; do
    IRT_PROBE_EXIT=$ex timeout -k 10 300 python3 profiles/rank_step.py --config $cfg --ranks 1,8 --modes frame --deals dealt \
      > $O/rank_${cfg}_exit$ex.jsonl 2> $O/rank_${cfg}_exit$ex.err || exit 1
  done
done
