# round 5 (e): scene-level miss-mode choice -- new terrain parity test, full GPU suite, benches
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "terrain or variants" -x -v -s --timeout 200 --timeout-method thread > $O/new_tests.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
for c in c3 c3t c5; do
  timeout -k 10 240 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
