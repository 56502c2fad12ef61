# round 4 (s): one-wave workgroups dealt so that a block's four packets share an XCD (workgroup
# i renders wave (i >> 3) & 3 of block ((i >> 5) << 3) | (i & 7)) against r04r's library
# (profiles/ablib/lib_wgsplit.so: consecutive workgroups = one block's waves, on four XCDs);
# the GPU suite first, then three interleaved rounds at C3, C3s, C4 (8 chained frames) and
# C5 (8 orbit views per launch)
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3 c3s c4 c5" $L profiles/ablib/lib_wgsplit.so || exit 1
