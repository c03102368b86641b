#!/bin/bash
# Round-5 baseline probes: the C2 call's per-chunk timeline (host timing), the C3 step by piece,
# and a rocprofv3 kernel trace of the C3 step (its HDR pass is the last call in the trace).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_base}
mkdir -p $O
cd $R
CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 4 > $O/host_timing_c2.log 2>&1 || { tail -20 $O/host_timing_c2.log; exit 1; }
timeout -k 10 200 python3 scripts/diag/c3_probe.py 10 > $O/c3_probe.log 2>&1 || { tail -20 $O/c3_probe.log; exit 1; }
CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python3 scripts/diag/c3_probe.py 2 > $O/c3_host_timing.log 2>&1 || { tail -20 $O/c3_host_timing.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_c3 -o run --output-format csv -- python3 $R/scripts/diag/c3_probe.py 2 > $O/trace_c3.log 2>&1 || { tail -20 $O/trace_c3.log; exit 1; }
python3 $R/scripts/diag/call_timeline.py $O/trace_c3 > $O/timeline_c3.txt
cat $O/c3_probe.log
tail -3 $O/host_timing_c2.log
