# round 4 (l): chained progressive frames -- the new tests and the progressive/tile tests, then
# C3 / C3s / C4 benches at 1, 2, 4, 8 frames per launch, and workgroup timelines of a chained launch
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chain.py \
  "tests/test_gpu_parity.py::test_progressive_batch_equals_sequential_frames" \
  tests/test_gpu_parity.py::test_tiles_accumulate_match_full_batch \
  tests/test_gpu_parity.py::test_dealt_tile_lists_match_full_frame > $O/tests.log 2>&1 || exit 1
for b in 1 2 4 8 16 1 2 4 8 16; do
  timeout -k 10 200 python3 bench.py --config c3 --batch $b --steps $((200 / b)) --warmup 3 --no-cpu-baseline >> $O/bench_c3.jsonl 2>> $O/bench.err || exit 1
done
for b in 1 4 1 4; do
  timeout -k 10 200 python3 bench.py --config c3s --batch $b --steps $((40 / b)) --warmup 2 --no-cpu-baseline >> $O/bench_c3s.jsonl 2>> $O/bench.err || exit 1
done
for b in 1 4 8; do
  timeout -k 10 200 python3 bench.py --config c4 --batch $b --steps $((80 / b)) --warmup 2 --no-cpu-baseline >> $O/bench_c4.jsonl 2>> $O/bench.err || exit 1
done
