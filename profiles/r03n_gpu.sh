# round 3 (n): kernel-argument tuples (load/store vectorizer off) x division forms, A/B
set -o pipefail
mkdir -p gpurun_out/r03n
L=profiles/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03n/gpu_tests.log 2>&1 || exit 1
bash profiles/ab_multi.sh gpurun_out/r03n/ab "c3 c3s" $L/lib_nodiv.so $L/lib_nodiv_nolsv.so $L/lib_div_nolsv.so $L/lib_recipcls_nolsv.so $L/lib_recip_nolsv.so
