# round 3 (q): uniform floats as kernel arguments (fewer VGPR constants), the 5-wave floor
# again, and the cooperative loop's speculation ramp re-tuned
set -o pipefail
mkdir -p gpurun_out/r03q
L=profiles/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03q/gpu_tests.log 2>&1 || exit 1
bash profiles/ab_multi.sh gpurun_out/r03q/ab "c3 c3s" $L/lib_p4_nolsv.so $L/lib_cf.so $L/lib_cf.so@IRT_RENDER_VARIANT=5376 $L/lib_cf.so@IRT_COOP_MAXLG=1 $L/lib_cf.so@IRT_COOP_RAMP=2
