# round 4 (zg): tile-list sequences (irt_render_tile_list_sequence) -- the chain tests, the
# 2-rank HIP split tests, a 2-rank gloo rehearsal of the C5-style orbit bench path on one GPU
# (small config C2 with the orbit camera is not defined: C5 itself, frame mode, 3 steps); then
# r04zf's six-wave A/B
set -o pipefail
O=gpurun_out/r04zg
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_chain.py \
  tests/test_gpu_distributed.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29535 bench.py --config c5 --gpus 2 --steps 3 --warmup 1 --mode frame --dist-backend gloo \
  > $O/bench_c5_dist2_frame.json 2> $O/bench_c5_dist2.err || exit 1
bash profiles/r04zf_gpu.sh || exit 1
