# round 4 (ze): the chained hand-off's write-through stores and loads with the streaming hint
# too (nt sc1, profiles/ablib/lib_ntsc1.so) against sc1 alone; chain tests on it first, then
# three interleaved rounds at C3, C3s, C4, C5 (8 frames / views per launch)
set -o pipefail
O=gpurun_out/r04ze
mkdir -p $O
L=icon-ray-tracing_amd/libicon_rt_hip.so
N=profiles/ablib/lib_ntsc1.so
IRT_LIB_PATH=$N timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chain.py > $O/tests_ntsc1.log 2>&1 || exit 1
ROUNDS=3 bash profiles/ab_multi.sh $O/ab "c3 c3s c4 c5" $L $N || exit 1
