# round 3 (l): full GPU suite + smoke on the round-3 kernel; wrap_coord fast path A/B vs HEAD
set -o pipefail
mkdir -p gpurun_out/r03l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03l/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03l/smoke.log 2>&1 || exit 1
bash profiles/ab_libs.sh gpurun_out/r03l/ab profiles/ab/libicon_rt_hip_base.so c3 c5
