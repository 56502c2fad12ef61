# round 3 (r): the prologue/setup VALU trims (constexpr LCG jump table, host-side lerp weight,
# scalar tile arithmetic, per-lane quotients through a refined double reciprocal) -- full GPU
# suite, smoke, A/B vs HEAD's build, the default bench line, rocprofv3 stats + PMC at C3
set -o pipefail
mkdir -p gpurun_out/r03r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r/smoke.log 2>&1 || exit 1
bash profiles/ab_libs.sh gpurun_out/r03r/ab profiles/ab/libicon_rt_hip_base.so c3 c3s c5 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03r/bench.json 2> gpurun_out/r03r/bench.err || exit 1
bash profiles/run_profiles.sh r03r_c3 --config c3 > /dev/null 2>&1 || exit 1
