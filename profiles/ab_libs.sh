#!/bin/bash
# profiles/ab_libs.sh OUT LIB_B [configs...]: bench.py with the in-tree library (A) and
# another build (B, via IRT_LIB_PATH) interleaved A B A B A B on one box, per config.
set -o pipefail
OUT=${1:?out}; LIBB=${2:?lib}; shift 2
CONFIGS=${@:-c3 c5}
mkdir -p "$OUT"
for cfg in $CONFIGS; do
  steps=200; [ "$cfg" = c5 ] && steps=60; [ "$cfg" = c3s ] && steps=40; [ "$cfg" = c4 ] && steps=80
  for round in 1 2 3; do
    timeout -k 10 240 python3 bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline --secondary none \
      >> "$OUT/A_$cfg.jsonl" 2>> "$OUT/A_$cfg.err" || exit 1
    IRT_LIB_PATH="$LIBB" timeout -k 10 240 python3 bench.py --config $cfg --steps $steps --warmup 5 \
      --no-cpu-baseline --secondary none >> "$OUT/B_$cfg.jsonl" 2>> "$OUT/B_$cfg.err" || exit 1
  done
done
