#!/bin/bash
# C1-shape call: path counts and a per-launch trace of every chunk; kernel stats under rocprofv3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_c1}
mkdir -p $O
cd $R
AB_COUNTS=1 CRISPR_NW_TRACE=8 CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 1 c1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -v "^nw host" $O/trace.log | tail -75
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o c1 --output-format csv -- python3 $R/scripts/diag/ab_call.py "" "" 3 c1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
cut -d, -f1-8 $O/kernel_stats.csv | head -20
