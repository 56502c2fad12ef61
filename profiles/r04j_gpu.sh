# round 4 (j), after the container was re-created: the full GPU suite on the current tree
# (slow-marked whole-frame tests included), smoke, the default bench, and r04i's OPT_PAIR A/B
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
LA=icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3s c3 c5" $L $LA@IRT_RENDER_VARIANT=268440832 || exit 1
