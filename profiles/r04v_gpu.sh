# round 4 (v): frames per launch 8 / 16 / 32 (bench.py --batch) on the shipped build, C3 and C3s,
# three interleaved rounds
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
for r in 1 2 3; do
  for b in 8 16 32; do
    for cfg in c3 c3s; do
      steps=$((1600 / b)); [ $cfg = c3s ] && steps=$((160 / b))
      timeout -k 10 240 python3 bench.py --config $cfg --batch $b --steps $steps --warmup 2 --no-cpu-baseline \
        --no-single-compare >> $O/b${b}_$cfg.jsonl 2>> $O/bench.err || exit 1
    done
  done
done
