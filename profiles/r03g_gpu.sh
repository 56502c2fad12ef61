# round 3 (g): where the fixed per-launch cost goes (IRT_PROBE_EXIT early returns)
set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 500 python3 profiles/probe.py --config c3 --rounds 5 --frames 20 --cases 'cam=away;IRT_PROBE_EXIT=1;IRT_PROBE_EXIT=2;IRT_PROBE_EXIT=3;IRT_PROBE_EXIT=1,IRT_COUNTERS=off;IRT_PROBE_EXIT=2,IRT_COUNTERS=off;IRT_PROBE_EXIT=3,IRT_COUNTERS=off;cam=away,IRT_COUNTERS=device;base;IRT_COUNTERS=device' > gpurun_out/r03g/probe_c3.jsonl 2> gpurun_out/r03g/probe_c3.err
