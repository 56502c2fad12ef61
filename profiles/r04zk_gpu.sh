# round 4 (zk): rocprofv3 kernel trace + FETCH/WRITE/L2 PMC passes of the final tree's bench,
# C3, C3s, C4 and C5 at the default 8 frames per launch
set -o pipefail
for c in c3 c3s c4 c5; do
  timeout -k 10 1000 bash profiles/run_profiles.sh r04zk_$c --config $c > /dev/null || exit 1
done
