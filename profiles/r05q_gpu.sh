#!/bin/bash
# round 5 (q): rocprofv3 kernel trace + FETCH/WRITE/L2 passes of the default kernel (LDS-DMA
# prologue, DPP prefix: 73405728 / 73667872) per config, the GPU suite, smoke and the bench line
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
for cfg in c3 c3s c5 c3t c4; do
  timeout -k 10 600 bash profiles/run_profiles.sh r05q_$cfg --config $cfg > $O/prof_$cfg.log 2>&1 || exit 1
done
timeout -k 10 600 bash profiles/run_profiles.sh r05q_c3b1 --config c3 --batch 1 > $O/prof_c3b1.log 2>&1 || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3 --launches 2 > $O/wg_c3_b1.jsonl 2> $O/wg_c3_b1.err || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_c3_full.json 2> $O/bench_c3_full.err || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
