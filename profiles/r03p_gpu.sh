# round 3 (p): getValue's path worked out once per sample (not per candidate test): parity,
# A/B against HEAD and the LDS-vector build, and the SQ instruction mix of each
set -o pipefail
mkdir -p gpurun_out/r03p
L=profiles/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03p/gpu_tests.log 2>&1 || exit 1
bash profiles/ab_multi.sh gpurun_out/r03p/ab "c3 c3s c5" $L/lib_div.so $L/lib_p4_nolsv.so $L/lib_pp_nolsv.so || exit 1
bash profiles/pmc_mix.sh gpurun_out/r03p/pmc $L/lib_div.so $L/lib_p4_nolsv.so $L/lib_pp_nolsv.so > gpurun_out/r03p/pmc_mix.txt 2>&1
