# round 3 (z): A/B on one box -- the previous HEAD build (abl/lib_head.so), the slot-done
# events without timestamps (abl/lib_evdt.so = the in-tree build), and two wave-priority
# builds on top of it: s_setprio 2 during the cooperative rounds / 0 for per-lane setup
# (abl/lib_prio.so) and the inverse (abl/lib_prioinv.so)
set -o pipefail
mkdir -p gpurun_out/r03z
bash profiles/ab_multi.sh gpurun_out/r03z/ab "c3 c4 c5" abl/lib_head.so abl/lib_evdt.so abl/lib_prio.so abl/lib_prioinv.so || exit 1
