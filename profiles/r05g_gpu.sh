# round 5 (g): the shipped kernels (miss mode on scenes with holes, its hole-free form on flat
# grids) -- rocprofv3 kernel trace + FETCH/WRITE/L2 passes per config, workgroup timelines,
# and the default bench line with its CPU baselines
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
for cfg in c3 c3s c5 c3t c4; do
  timeout -k 10 600 bash profiles/run_profiles.sh r05g_$cfg --config $cfg > $O/prof_$cfg.log 2>&1 || exit 1
done
timeout -k 10 600 bash profiles/run_profiles.sh r05g_c3b1 --config c3 --batch 1 > $O/prof_c3b1.log 2>&1 || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3 --launches 2 > $O/wg_c3_b1.jsonl 2> $O/wg_c3_b1.err || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3 --launches 2 --batch 8 > $O/wg_c3_b8.jsonl 2> $O/wg_c3_b8.err || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_c3_full.json 2> $O/bench_c3_full.err || exit 1
