#!/bin/bash
# profiles/ab_multi.sh OUT "CONFIGS" LIB[@VAR=VAL[@VAR=VAL]]... : bench.py with each library
# (IRT_LIB_PATH) and its environment overrides, round-robin, $ROUNDS rounds (default 3), on one box;
# OUT/<lib-basename>[_<VAL>...]_<cfg>.jsonl.
set -o pipefail
OUT=${1:?out}; CONFIGS=${2:?configs}; shift 2
mkdir -p "$OUT"
for cfg in $CONFIGS; do
  # frames per run as before round 4's chained batches; BATCH frames per launch (bench.py --batch)
  B=${BATCH:-8}
  steps=200; [ "$cfg" = c5 ] && steps=60; [ "$cfg" = c3s ] && steps=40; [ "$cfg" = c4 ] && steps=80
  steps=$(( (steps + B - 1) / B ))
  for round in $(seq 1 ${ROUNDS:-3}); do
    for spec in "$@"; do
      IFS=@ read -r lib envs <<< "$spec"
      n=$(basename "$lib" .so)
      vars=()
      if [ -n "$envs" ]; then
        IFS=@ read -r -a kv <<< "$envs"
        for a in "${kv[@]}"; do vars+=("$a"); v="${a#IRT_}"; [ "${a%%=*}" = IRT_RENDER_VARIANT ] && v="${a#*=}"; n="${n}_${v}"; done
      fi
      env IRT_LIB_PATH="$lib" "${vars[@]}" timeout -k 10 240 python3 bench.py --config $cfg --batch $B --steps $steps --no-single-compare \
        --warmup 5 --no-cpu-baseline --secondary none >> "$OUT/${n}_$cfg.jsonl" 2>> "$OUT/${n}_$cfg.err" || exit 1
    done
  done
done
