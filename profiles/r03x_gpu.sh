# round 3 (x): per-step overhead outside the kernel -- the statistics' per-workgroup stores into
# pinned host memory vs device memory vs none (IRT_COUNTERS, measurement only), with the bench's
# timed launches cut to four per run; then the default bench line
set -o pipefail
mkdir -p gpurun_out/r03x
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03x/ab "c3 c4" $L $L@IRT_COUNTERS=device $L@IRT_COUNTERS=off || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03x/bench.json 2> gpurun_out/r03x/bench.err || exit 1
