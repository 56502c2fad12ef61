# round 4 (h), r04g's content again (its first try found a stale library) and OPT_NEXTHDR:
# - smoke; bench.py with per-launch statistics off in the timed loop (the new default; counts
#   from re-rendering the same steps) and on;
# - every A/B variant bit-identical on the A/B library;
# - interleaved, C3s and C3: the cooperative loop's speculation ramp (IRT_COOP_RAMP 2 / 3,
#   IRT_COOP_MAXLG 2) and OPT_NEXTHDR (134223104: each solo round after a wave's first also
#   loads the header line of the ray's next sample) against the default; C5: OPT_NEXTHDR;
# - C5's translation and L1->L2 latency counters (C3/C3s in profiles/r04d_pmc/)
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 bench.py --stats on --no-cpu-baseline > $O/bench_stats_on.json 2> $O/bench_stats_on.err || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 360 --timeout-method thread \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/variants.log 2>&1 || exit 1
ROUNDS=2 bash profiles/ab_multi.sh $O/ab "c3s c3" $L $L@IRT_COOP_RAMP=2 $L@IRT_COOP_RAMP=3 $L@IRT_COOP_MAXLG=2 \
  $LA@IRT_RENDER_VARIANT=134223104 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab c5 $L $LA@IRT_RENDER_VARIANT=134223104 || exit 1
bash profiles/pmc_latency.sh r04h_c5 --config c5 > $O/pmclat_c5.log 2>&1
