# round 5 (f): compact certified entries -- full GPU suite, then the tree against the
# pre-compact library (miss mode in both), interleaved on one box
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
ROUNDS=2 timeout -k 10 900 bash profiles/ab_multi.sh $O/ab "c3 c3t c3s c5" $PWD/icon-ray-tracing_amd/libicon_rt_hip.so $PWD/profiles/ablib/lib_r05_missmode.so > $O/ab.log 2>&1 || exit 1
