# round 5 (b): the new chain / RCCL / terrain tests, the full GPU suite, C3t bench + profile
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_chain.py tests/test_gpu_distributed.py -x -v -s --timeout 120 --timeout-method thread > $O/new_tests.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --config c3t --no-cpu-baseline > $O/bench_c3t.json 2> $O/bench_c3t.err || exit 1
timeout -k 10 600 bash profiles/run_profiles.sh r05b_c3t --config c3t > $O/prof_c3t.log 2>&1 || exit 1
