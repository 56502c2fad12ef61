# round 4 (h): OPT_NEXTHDR (134223104: each solo round after a wave's first also loads the
# header line of the ray's next sample) -- every A/B variant bit-identical on the A/B
# library, then interleaved against the default of the same library at C3s, C3, C5
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 360 --timeout-method thread \
  tests/test_gpu_parity.py::test_ab_library_variants_identical > $O/variants.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3s c3 c5" $LA $LA@IRT_RENDER_VARIANT=134223104 || exit 1
# C5's translation and L1->L2 latency counters (C3/C3s in profiles/r04d_pmc/)
bash profiles/pmc_latency.sh r04h_c5 --config c5 > $O/pmclat_c5.log 2>&1
