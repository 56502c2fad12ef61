set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "variants or scheduling or progressive or tiles" > gpurun_out/gpu_tests3.log 2>&1
for rep in 1 2; do
for v in 5120 70656 69632 70912; do
for sc in 1 0; do
IRT_SCHED=$sc IRT_RENDER_VARIANT=$v timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline > gpurun_out/ab_v$v.s$sc.json 2>/dev/null
echo "v=$v sched=$sc $(python3 -c "import json;d=json.load(open('gpurun_out/ab_v$v.s$sc.json'));print(d['ms_per_step'],d['config']['kernel_ms_rank0'])")"
done; done; done
tail -2 gpurun_out/gpu_tests3.log
