# round 4 (zb): the multi-rank bench path on the final build, rehearsed with two gloo ranks on
# one GPU (progressive and frame mode), and the C++ app's bench with the true-size camera
set -o pipefail
O=gpurun_out/r04zb
mkdir -p $O
for mode in progressive frame; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29534 bench.py --gpus 2 --steps 10 --warmup 2 --mode $mode --dist-backend gloo \
    > $O/bench_dist2_$mode.json 2> $O/bench_dist2_$mode.err || exit 1
done
for b in 1 8; do
  timeout -k 10 200 icon-ray-tracing_amd/icon_rt --synth 2 7 90 --size 1024 1024 --camera 0 0 1.4e7 0 0 0 0 1 0 \
    -fovy 60 --true-size --sample-limit 1 --bench 800 --frames-per-launch $b >> $O/icon_rt_bench.txt 2>&1 || exit 1
done
