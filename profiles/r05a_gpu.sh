# round 5 (a): baseline of the round-4 tree on this round's boxes -- C3, C3s, C5 bench lines
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
for c in c3 c3s c5; do
  timeout -k 10 240 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
