set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "variants" > gpurun_out/gpu_tests8.log 2>&1
for cfg in c3 c4; do
for rep in 1 2; do
for v in 5120 70656 136192 136448; do
IRT_RENDER_VARIANT=$v timeout -k 10 200 python bench.py --config $cfg --steps 300 --no-cpu-baseline > gpurun_out/ab_$cfg.v$v.json 2>/dev/null
echo "$cfg v=$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$cfg.v$v.json'));print(d['ms_per_step'],d['config']['kernel_ms_rank0'])")"
done; done; done
tail -2 gpurun_out/gpu_tests8.log
