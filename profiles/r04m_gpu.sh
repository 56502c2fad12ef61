# round 4 (m): chained frames as the bench default (--batch 8): smoke, the full GPU suite, the
# default bench (CPU baseline included), a 2-rank rehearsal of the multi-GPU progressive path
# on one GPU (gloo), rocprofv3 kernel stats + FETCH/WRITE/L2 PMC passes at C3 (batch 8 and 1),
# C3s (batch 4), C5 (orbit: one frame per launch), and the chained launch's workgroup timeline
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --dist-backend gloo > $O/bench_dist2_gloo.json 2> $O/bench_dist2.err || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04m_c3 --config c3 > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04m_c3b1 --config c3 --batch 1 > $O/prof_c3b1.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04m_c3s --config c3s --batch 4 --steps 5 > $O/prof_c3s.log 2>&1 || exit 1
timeout -k 10 400 bash profiles/run_profiles.sh r04m_c5 --config c5 > $O/prof_c5.log 2>&1 || exit 1
