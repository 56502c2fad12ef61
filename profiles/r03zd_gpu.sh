# round 3 (zd): streaming stores of the per-frame samples in progressive batches (the N>1
# bench's launches), A/B on one box with profiles/rank_step.py (every rank's share at N = 2, 8)
set -o pipefail
mkdir -p gpurun_out/r03zd
for cfg in c3 c4; do
  for round in 1 2 3; do
    for lib in abl/lib_cur.so abl/lib_ntsamp.so; do
      n=$(basename $lib .so)
      IRT_LIB_PATH=$lib timeout -k 10 300 python3 profiles/rank_step.py --config $cfg --ranks 2,8 \
        --modes progressive --deals dealt --steps 40 >> gpurun_out/r03zd/${n}_$cfg.jsonl 2>> gpurun_out/r03zd/${n}_$cfg.err || exit 1
    done
  done
done
