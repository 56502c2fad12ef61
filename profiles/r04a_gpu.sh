# round 4 (a): the round's first GPU pass: smoke, the whole GPU suite (slow C2-C5 whole-frame
# parity included; value[31] grid build, persistent launches, the certified fast lat/lon and
# its exhaustive bounds), the default bench line, and the C3 decomposition -- IRT_PROBE_EXIT
# stops, per-region shader clocks of the 5-wave timing variant, the persistent launch, the
# lean-LDS 6-wave build (80 VGPRs), the 4-wave build
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
IRT_LIB_PATH=icon-ray-tracing_amd/libicon_rt_hip_all.so timeout -k 10 600 python3 profiles/probe.py --config c3 --rounds 3 --frames 20 \
  --cases 'base;IRT_QUEUE=1;IRT_PROBE_EXIT=3;IRT_PROBE_EXIT=4;IRT_PROBE_EXIT=5;variant=529664;variant=2102784;variant=2102528;variant=5120;tf=comb;tf=comb,IRT_QUEUE=1;tf=comb,variant=529664;tf=comb,variant=2102784' \
  > $O/probe_c3.jsonl 2> $O/probe_c3.err || exit 1
