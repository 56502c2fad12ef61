set -e
mkdir -p gpurun_out
for cfg in c3 c4; do
for rep in 1 2; do
for sc in 1 2 3 0; do
IRT_SCHED=$sc timeout -k 10 200 python bench.py --config $cfg --steps 300 --no-cpu-baseline > gpurun_out/ab3_$cfg.s$sc.json 2>/dev/null
echo "$cfg sched=$sc $(python3 -c "import json;d=json.load(open('gpurun_out/ab3_$cfg.s$sc.json'));print(d['ms_per_step'],d['config']['kernel_ms_rank0'])")"
done; done; done
