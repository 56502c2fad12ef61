# round 4 (d): rocprofv3 kernel-trace stats + FETCH/WRITE/L2 PMC passes of the shipped build
# at C3, C3s and C5 (profiles/run_profiles.sh), the SQ instruction mix against the round-3
# kernel, and the address/latency counters at C3s and C3
set -o pipefail
mkdir -p gpurun_out/r04d
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/run_profiles.sh r04d_c3 --config c3 > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r04d_c3s --config c3s > /dev/null 2>&1 || exit 1
bash profiles/run_profiles.sh r04d_c5 --config c5 > /dev/null 2>&1 || exit 1
bash profiles/pmc_mix.sh gpurun_out/r04d/mix $L ab/lib_base.so > gpurun_out/r04d/mix.txt 2>&1 || exit 1
bash profiles/pmc_latency.sh r04d_c3s --config c3s > /dev/null 2>&1 || exit 1
bash profiles/pmc_latency.sh r04d_c3 --config c3 > /dev/null 2>&1 || exit 1
