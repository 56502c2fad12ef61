# round 5 (c): C3t after the inverted-first-layer meta fix -- bench (8 and 1 frames per
# launch), workgroup timeline of single frames, region clocks and statistics (A/B library)
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 240 python3 bench.py --config c3t --no-cpu-baseline > $O/bench_c3t.json 2> $O/bench_c3t.err || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 3 > $O/wg_c3t_b1.jsonl 2> $O/wg_c3t_b1.err || exit 1
timeout -k 10 180 python3 profiles/wg_trace.py --config c3 --launches 2 > $O/wg_c3_b1.jsonl 2> $O/wg_c3_b1.err || exit 1
export IRT_LIB_PATH=$PWD/icon-ray-tracing_amd/libicon_rt_hip_all.so
timeout -k 10 300 python3 profiles/probe.py --config c3t --cases 'base;variant=36864;variant=529664' --rounds 2 > $O/probe_c3t.jsonl 2> $O/probe_c3t.err || exit 1
timeout -k 10 300 python3 profiles/probe.py --config c3 --cases 'base;variant=36864;variant=529664' --rounds 2 > $O/probe_c3.jsonl 2> $O/probe_c3.err || exit 1
