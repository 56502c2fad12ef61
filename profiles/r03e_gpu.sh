# round 3 (e): shell build rewrite, lazy grid, counter fixes -- tests + C5 creation stages
set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grid.py tests/test_gpu_build.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e/gpu_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for cfg in "2 7 90" "2 9 90"; do
  IRT_BUILD_VERBOSE=1 timeout -k 10 300 python3 -c "
import sys, time; sys.path.insert(0, '$GRAFT_REPO_ROOT/icon-ray-tracing_amd/python')
import irt
t = time.time(); c = irt.Context.synth($(echo $cfg | tr ' ' ','), 0); print('create', round(time.time() - t, 3), 's', c.info.deviceBytes / 2**30, 'GiB', flush=True)
" >> $GRAFT_REPO_ROOT/gpurun_out/r03e/create.txt 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03e/create_c5 -o run -- python3 -c "
import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT/icon-ray-tracing_amd/python')
import irt
c = irt.Context.synth(2, 9, 90, 0)
" > $GRAFT_REPO_ROOT/gpurun_out/r03e/create_c5_prof.log 2>&1
