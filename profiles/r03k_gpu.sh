# round 3 (k): loop-invariant uniforms recomputed per call (asm barriers) vs HEAD; 5-wave floor
set -o pipefail
mkdir -p gpurun_out/r03k
timeout -k 10 300 python3 profiles/probe.py --config c3 --rounds 6 --frames 20 --cases 'base;variant=5376;tf=comb;tf=comb,variant=5376' > gpurun_out/r03k/probe_c3.jsonl 2> gpurun_out/r03k/probe_c3.err || exit 1
IRT_LIB_PATH=profiles/ab/libicon_rt_hip_base.so timeout -k 10 300 python3 profiles/probe.py --config c3 --rounds 6 --frames 20 --cases 'base;tf=comb' > gpurun_out/r03k/probe_c3_head.jsonl 2> gpurun_out/r03k/probe_c3_head.err || exit 1
timeout -k 10 300 python3 profiles/probe.py --config c3 --rounds 6 --frames 20 --cases 'base;tf=comb' > gpurun_out/r03k/probe_c3_again.jsonl 2> gpurun_out/r03k/probe_c3_again.err
