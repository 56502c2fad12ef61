# round 3 (f): C5 shell build after LDS staging; fixed-cost probe cases at C3
set -o pipefail
mkdir -p gpurun_out/r03f
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03f/create_c5 -o run -- python3 -c "
import sys; sys.path.insert(0, '$R/icon-ray-tracing_amd/python')
import irt
c = irt.Context.synth(2, 9, 90, 0)
" > $R/gpurun_out/r03f/create_c5_prof.log 2>&1 || exit 1
cd $R
timeout -k 10 500 python3 profiles/probe.py --config c3 --rounds 5 --frames 20 --cases 'base;IRT_COUNTERS=off;cam=away;cam=away,IRT_COUNTERS=off;tf=dense;tf=zero;variant=36864;IRT_COOP_MAXLG=1;IRT_COOP_RAMP=2' > gpurun_out/r03f/probe_c3.jsonl 2> gpurun_out/r03f/probe_c3.err
