# round 4 (u): one-wave workgroups with the accum pixel prefetched into LDS at the ray's start
# (1 KB more LDS per workgroup: 7,992 B) against loading it at the end (profiles/ablib/
# lib_accend.so, r04t's build); the chain and parity tests first, then three interleaved rounds
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chain.py \
  tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3 c3s c4 c5" $L profiles/ablib/lib_accend.so || exit 1
