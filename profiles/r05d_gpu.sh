# round 5 (d): the miss mode in the default kernel -- parity (chain, parity, scale suites),
# C3t / C3 / C3s / C5 bench lines, and an in-process A/B of the miss mode (OPT_NOMISS)
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
for c in c3t c3 c3s c5; do
  timeout -k 10 240 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
timeout -k 10 180 python3 profiles/wg_trace.py --config c3t --launches 2 > $O/wg_c3t_b1.jsonl 2> $O/wg_c3t_b1.err || exit 1
export IRT_LIB_PATH=$PWD/icon-ray-tracing_amd/libicon_rt_hip_all.so
for c in c3 c3t; do
  timeout -k 10 300 python3 profiles/probe.py --config $c --cases 'base;variant=6558976;base;variant=6558976;variant=36864' --rounds 3 > $O/probe_$c.jsonl 2> $O/probe_$c.err || exit 1
done
