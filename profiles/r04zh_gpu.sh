# round 4 (zh): the final tree -- smoke, the full GPU suite, the default bench (CPU baseline
# included), C5 with 8 orbit views per launch, and a 2-rank gloo rehearsal of the progressive
# orbit split (irt_render_tile_list_sequence) on one GPU
set -o pipefail
O=gpurun_out/r04zh
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29536 bench.py --config c5 --gpus 2 --steps 5 --warmup 1 --dist-backend gloo \
  > $O/bench_c5_dist2_progressive.json 2> $O/bench_c5_dist2.err || exit 1
