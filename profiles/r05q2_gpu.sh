#!/bin/bash
# round 5 (q, second part): the GPU suite and smoke on the final tree (the A/B library now
# lists the default variant), then the measured-cost order A/B (profiles/r05r_gpu.sh)
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
bash profiles/r05r_gpu.sh || exit 1
