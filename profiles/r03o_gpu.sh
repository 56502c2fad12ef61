# round 3 (o): LDS slots as explicit 16-byte vectors, with / without the IR load/store vectorizer
set -o pipefail
mkdir -p gpurun_out/r03o
L=profiles/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03o/gpu_tests.log 2>&1 || exit 1
bash profiles/ab_multi.sh gpurun_out/r03o/ab "c3 c3s" $L/lib_div.so $L/lib_div_nolsv.so $L/lib_p4_lsv.so $L/lib_p4_nolsv.so $L/lib_nodiv.so
