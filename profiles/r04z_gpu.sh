# round 4 (z): the final tree -- smoke, the full GPU suite, the default bench (CPU baseline
# included), the C++ icon_rt app's bench at 1 and 8 frames per launch (R2B07 x 90, 1024^2)
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
for b in 1 8; do
  timeout -k 10 200 icon-ray-tracing_amd/icon_rt --synth 2 7 90 --size 1024 1024 --camera 0 0 1.4e7 0 0 0 0 1 0 \
    -fovy 60 --sample-limit 1 --bench 400 --frames-per-launch $b >> $O/icon_rt_bench.txt 2>&1 || exit 1
done
