# round 4 (za): instruction mix and memory-pipeline counters of the shipped kernel at C3 with 8
# chained frames per launch (one rocprofv3 --pmc pass per counter group), and the C++ icon_rt
# app's bench at 1 and 8 frames per launch (launches back to back, counting off)
set -o pipefail
O=gpurun_out/r04za
mkdir -p $O
CONFIG=c3 timeout -k 10 200 bash profiles/pmc_mix.sh gpurun_out/r04za/mix icon-ray-tracing_amd/libicon_rt_hip.so > $O/mix.txt 2>&1 || exit 1
timeout -k 10 400 bash profiles/pmc_latency.sh r04za_c3 --config c3 > $O/latency_c3.txt 2>&1 || exit 1
for b in 1 8; do
  timeout -k 10 200 icon-ray-tracing_amd/icon_rt --synth 2 7 90 --size 1024 1024 --camera 0 0 1.4e7 0 0 0 0 1 0 \
    -fovy 60 --sample-limit 1 --bench 800 --frames-per-launch $b >> $O/icon_rt_bench.txt 2>&1 || exit 1
done
