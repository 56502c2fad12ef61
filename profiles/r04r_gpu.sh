# round 4 (r): orbit sequences in one launch (irt_render_sequence) and the bucketed count
# fallback: the full GPU suite, smoke, the default bench, C5 benches at 1 and 8 orbit views per
# launch, rocprofv3 + PMC at C4 (8 chained frames) and C5 (8 views per launch), every rank's
# share at C4 (statistics off, as bench.py's timed loop)
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
for b in 1 8 1 8; do
  timeout -k 10 300 python3 bench.py --config c5 --batch $b --steps $((120 / b)) --warmup 2 --no-cpu-baseline >> $O/bench_c5.jsonl 2>> $O/bench_c5.err || exit 1
done
timeout -k 10 400 bash profiles/run_profiles.sh r04r_c4 --config c4 --steps 5 > $O/prof_c4.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04r_c5 --config c5 --steps 10 > $O/prof_c5.log 2>&1 || exit 1
timeout -k 10 400 python3 profiles/rank_step.py --config c4 --batch 8 --deals dealt --steps 20 > $O/rank_c4_b8.jsonl 2> $O/rank_c4.err || exit 1
