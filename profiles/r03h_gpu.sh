# round 3 (h): two-tasks-per-lane candidate deal (default) vs round-2 first-candidate scan
set -o pipefail
mkdir -p gpurun_out/r03h
# (parity: 29 passed on the first run)
timeout -k 10 500 python3 profiles/probe.py --config c3 --rounds 6 --frames 20 --cases 'base;variant=267264;variant=4096;tf=comb;tf=comb,variant=267264;tf=dense;tf=dense,variant=267264' > gpurun_out/r03h/probe_c3.jsonl 2> gpurun_out/r03h/probe_c3.err
