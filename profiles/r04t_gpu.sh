# round 4 (t): the shipped build (one-wave workgroups dealt per XCD, chained frames, orbit
# sequences): smoke, the default bench, rocprofv3 kernel stats + FETCH/WRITE/L2 PMC passes at C3
# (8 chained frames and 1), C3s, C4 (8), C5 (8 orbit views per launch), the chained launch's
# workgroup timeline at C3
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04t_c3 --config c3 > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04t_c3b1 --config c3 --batch 1 > $O/prof_c3b1.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04t_c3s --config c3s --steps 3 > $O/prof_c3s.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04t_c4 --config c4 --steps 5 > $O/prof_c4.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04t_c5 --config c5 --steps 10 > $O/prof_c5.log 2>&1 || exit 1
timeout -k 10 200 python3 profiles/wg_trace.py --config c3 --batch 8 --launches 2 > $O/wg_trace_c3_b8.jsonl 2> $O/wg_trace.err || exit 1
