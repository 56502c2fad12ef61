# round 3: per-rank shares of the multi-GPU step (profiles/rank_step.py), C3 and C4
set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 400 python -u profiles/rank_step.py --config c3 --steps 40 > gpurun_out/r03c/rank_step_c3.jsonl 2> gpurun_out/r03c/rank_step_c3.err && \
timeout -k 10 400 python -u profiles/rank_step.py --config c4 --steps 20 > gpurun_out/r03c/rank_step_c4.jsonl 2> gpurun_out/r03c/rank_step_c4.err
