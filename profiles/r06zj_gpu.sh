#!/bin/bash
# round 6 (zj): bench.py --gpus 4 and 8 over gloo on the one GPU (the scaling run's deal, launcher and
# assembled frame), the bench tests
set -o pipefail
O=gpurun_out/r06zj
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_bench.py > $O/tests_bench.log 2>&1 || exit 1
