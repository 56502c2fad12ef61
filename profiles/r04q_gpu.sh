# round 4 (q): one-wave workgroups as the default (6296832): smoke, the full GPU suite, the
# default bench, rocprofv3 kernel stats + FETCH/WRITE/L2 PMC at C3 (8 chained frames and 1),
# C3s (8), C4 (8), C5 (orbit), the chained launch's timeline, and every rank's share at 8
# chained frames per launch (C3, C4)
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04q_c3 --config c3 > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04q_c3b1 --config c3 --batch 1 > $O/prof_c3b1.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04q_c3s --config c3s --steps 3 > $O/prof_c3s.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04q_c4 --config c4 --steps 5 > $O/prof_c4.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04q_c5 --config c5 > $O/prof_c5.log 2>&1 || exit 1
timeout -k 10 200 python3 profiles/wg_trace.py --config c3 --batch 8 --launches 2 > $O/wg_trace_c3_b8.jsonl 2> $O/wg_trace.err || exit 1
for cfg in c3 c4; do
  timeout -k 10 400 python3 profiles/rank_step.py --config $cfg --batch 8 --deals dealt --steps 20 > $O/rank_${cfg}_b8.jsonl 2> $O/rank_${cfg}.err || exit 1
done
