set -e
mkdir -p gpurun_out
IRT_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "variants or scheduling or progressive or tiles or bit_exact" > gpurun_out/gpu_tests4.log 2>&1
for rep in 1 2; do
for x in 0 1; do
for sc in 1 0 3; do
IRT_XCD=$x IRT_SCHED=$sc timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline > gpurun_out/ab_x$x.s$sc.json 2>/dev/null
echo "xcd=$x sched=$sc $(python3 -c "import json;d=json.load(open('gpurun_out/ab_x$x.s$sc.json'));print(d['ms_per_step'],d['config']['kernel_ms_rank0'])")"
done; done; done
tail -2 gpurun_out/gpu_tests4.log
