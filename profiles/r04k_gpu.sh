# round 4 (k): workgroup timelines (profiles/wg_trace.py: every workgroup's start/end and XCC)
# of back-to-back launches at C3, C3s, C4, C5 -- the ramp, the tail and the gaps between launches
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
for cfg in c3 c3s c4 c5; do
  timeout -k 10 240 python3 profiles/wg_trace.py --config $cfg --launches 4 > $O/wg_trace_$cfg.jsonl 2> $O/wg_trace_$cfg.err || exit 1
done
