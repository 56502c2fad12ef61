# round 4 (zi): every rank's share of the C5 orbit step at N = 1, 2, 4, 8 with 8 views per launch
# (irt_render_tile_list_sequence), timed on one GPU (profiles/rank_step.py)
set -o pipefail
O=gpurun_out/r04zi
mkdir -p $O
timeout -k 10 900 python3 -u profiles/rank_step.py --config c5 --batch 8 --steps 20 --deals dealt \
  > $O/rank_step_c5_b8.jsonl 2> $O/rank_step_c5_b8.err || exit 1
