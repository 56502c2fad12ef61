#!/bin/bash
# round 6 (g): what the end of a wave costs at one frame per launch (IRT_PROBE_EXIT=6: the lerp
# without its accum read; 7: no accum read and no pixel stores; measurement only, frames differ),
# C3 and C3t; the statistics variant's per-wave counts (rounds, locate rounds, entry hops) at C3
# and C3t; a workgroup timeline of C3t single frames
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 200 python3 profiles/probe.py --config c3 --cases "base;IRT_PROBE_EXIT=6;IRT_PROBE_EXIT=7;variant=36864" --rounds 3 > $O/probe_c3.jsonl 2> $O/probe_c3.err || exit 1
timeout -k 10 200 python3 profiles/probe.py --config c3t --cases "base;IRT_PROBE_EXIT=6;IRT_PROBE_EXIT=7;variant=36864" --rounds 3 > $O/probe_c3t.jsonl 2> $O/probe_c3t.err || exit 1
timeout -k 10 200 python3 profiles/wg_trace.py --config c3t --batch 1 --launches 3 > $O/wg_c3t_b1.jsonl 2> $O/wg_c3t_b1.err || exit 1
