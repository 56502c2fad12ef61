# round 3 (w): one-wave workgroups (OPT_WAVEWG with OPT_LEAN: 7 KB of LDS per workgroup, a
# finished wave frees its slot at once) at 4 and 5 waves/SIMD; the cooperative loop's initial
# speculation at 5 waves; C4 frame-mode per-rank shares with the 5-wave default
set -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w/gpu_tests.log 2>&1 || exit 1
L=icon-ray-tracing_amd/libicon_rt_hip.so
bash profiles/ab_multi.sh gpurun_out/r03w/ab "c3 c4 c3s c5" $L@IRT_RENDER_VARIANT=5376 $L@IRT_RENDER_VARIANT=6296832 $L@IRT_RENDER_VARIANT=6296576 $L@IRT_RENDER_VARIANT=5376@IRT_COOP_MAXLG=1 || exit 1
timeout -k 10 400 python3 profiles/rank_step.py --config c4 --modes frame,progressive --deals dealt --ranks 1,2,4,8 > gpurun_out/r03w/rank_c4.jsonl 2> gpurun_out/r03w/rank_c4.err || exit 1
# SQ occupancy / instruction mix per variant (one --pmc pass each, 8 SQ counters, kernel trace only)
cd /tmp && export TMPDIR=/tmp
for v in 5376 5120 6296832; do
  IRT_RENDER_VARIANT=$v timeout -s KILL 120 rocprofv3 --kernel-trace \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r03w/pmc_$v" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline \
    > "$GRAFT_REPO_ROOT/gpurun_out/r03w/pmc_$v.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r03w/pmc_$v.err" || exit 1
done
