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
CONFIG=c3s bash profiles/pmc_mix.sh gpurun_out/r04d/mix_c3s $L > gpurun_out/r04d/mix_c3s.txt 2>&1 || exit 1
bash profiles/pmc_latency.sh r04d_c3s --config c3s > /dev/null 2>&1 || exit 1
bash profiles/pmc_latency.sh r04d_c3 --config c3 > /dev/null 2>&1 || exit 1
# every rank's share of a frame-mode (strong) step on one GPU: grid launch, persistent launch,
# whole-wave speculation from the first round
for cfg in c3 c4; do
  for envs in "" "IRT_QUEUE=1" "IRT_COOP_MAXLG=6"; do
    n=${envs:-base}; n=${n//=/_}
    env $envs timeout -k 10 300 python3 profiles/rank_step.py --config $cfg --modes frame --deals dealt \
      > gpurun_out/r04d/rank_${cfg}_$n.jsonl 2> gpurun_out/r04d/rank_${cfg}_$n.err || exit 1
  done
done
# the instruction mix of the launch stopped at successive points (IRT_PROBE_EXIT: 3 after ray
# generation and boxTest, 4 at the first woodcockFunc, 5 after it), C3 and C3s
for ex in 3 4 5; do
  IRT_PROBE_EXIT=$ex bash profiles/pmc_mix.sh gpurun_out/r04d/mix_exit$ex $L > gpurun_out/r04d/mix_exit$ex.txt 2>&1 || exit 1
  IRT_PROBE_EXIT=$ex CONFIG=c3s bash profiles/pmc_mix.sh gpurun_out/r04d/mix_c3s_exit$ex $L > gpurun_out/r04d/mix_c3s_exit$ex.txt 2>&1 || exit 1
done
