# round 4 (zn): the raygen's L2->fabric read requests by size and those served by DRAM rather
# than the Infinity Cache (profiles/calib/render_requests.sh), final tree, 8 frames per launch
set -o pipefail
for c in c3 c3s c4 c5; do
  timeout -k 10 500 bash profiles/calib/render_requests.sh $c > gpurun_out/req_$c.json || exit 1
done
