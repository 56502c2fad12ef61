# round 4 (g): bench.py with per-launch statistics off in the timed loop (the new default;
# counts from re-rendering the same steps) and on; smoke; the cooperative loop's speculation
# ramp for the comb TF (IRT_COOP_RAMP 2 / 3, IRT_COOP_MAXLG 2) against the default, C3s and C3
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 bench.py --stats on --no-cpu-baseline > $O/bench_stats_on.json 2> $O/bench_stats_on.err || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3s c3" $L $L@IRT_COOP_RAMP=2 $L@IRT_COOP_RAMP=3 $L@IRT_COOP_MAXLG=2 || exit 1
