#!/bin/bash
# profiles/run_profiles.sh TAG [bench args...]
# Runs on the GPU box (via gpurun) from the repo root.  Produces, under gpurun_out/prof_TAG:
#   stats/   rocprofv3 --kernel-trace --stats (CSV) of `bench.py --steps 20`
#   pmc_fetch/, pmc_write/, pmc_l2/   one --pmc pass each (counters never combined with
#            runtime/sys traces; FETCH_SIZE and WRITE_SIZE need separate passes on gfx950)
# then summarises them with profiles/summarize.py into gpurun_out/prof_TAG/summary.json.
set -euo pipefail
TAG=${1:?tag}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS=(--steps 20 --warmup 2 --no-cpu-baseline --no-single-compare --secondary none "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
  -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_stats.json" 2> "$OUT/bench_stats.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_l2" -o run \
  -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_l2.json" 2> "$OUT/bench_l2.err"
python3 "$ROOT/profiles/summarize.py" "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
