# round 4 (zj): bench.py reports chain_timeouts (single GPU and two gloo ranks on one GPU)
set -o pipefail
O=gpurun_out/r04zj
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 50 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29537 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo \
  > $O/bench_dist2.json 2> $O/bench_dist2.err || exit 1
