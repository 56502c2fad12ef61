# round 3 (i): LDS-staged shell build checks; where a C3 frame's time goes (IRT_PROBE_EXIT 3/4/5)
set -o pipefail
mkdir -p gpurun_out/r03i
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grid.py -m gpu -x -q --timeout 300 --timeout-method thread -k "shell or grid or counter" > gpurun_out/r03i/gpu_tests.log 2>&1 || exit 1
timeout -k 10 500 python3 profiles/probe.py --config c3 --rounds 5 --frames 20 --cases 'base;cam=away;IRT_PROBE_EXIT=3;IRT_PROBE_EXIT=4;IRT_PROBE_EXIT=5;tf=dense;tf=dense,IRT_PROBE_EXIT=4;tf=dense,IRT_PROBE_EXIT=5;tf=zero' > gpurun_out/r03i/probe_c3.jsonl 2> gpurun_out/r03i/probe_c3.err
