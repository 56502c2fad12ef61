# round 3 (j): XCD-aware workgroup -> block order (IRT_XCD_REMAP 0/1/2)
set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 500 python3 profiles/probe.py --config c3 --rounds 6 --frames 20 --cases 'IRT_XCD_REMAP=0;IRT_XCD_REMAP=1;IRT_XCD_REMAP=2;tf=comb,IRT_XCD_REMAP=0;tf=comb,IRT_XCD_REMAP=1;tf=comb,IRT_XCD_REMAP=2' > gpurun_out/r03j/probe_c3.jsonl 2> gpurun_out/r03j/probe_c3.err || exit 1
timeout -k 10 500 python3 profiles/probe.py --config c4 --rounds 4 --frames 10 --cases 'IRT_XCD_REMAP=0;IRT_XCD_REMAP=1;IRT_XCD_REMAP=2' > gpurun_out/r03j/probe_c4.jsonl 2> gpurun_out/r03j/probe_c4.err
