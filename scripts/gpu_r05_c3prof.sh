#!/bin/bash
# C3 step by piece and its kernels' time (rocprofv3 kernel stats of 3 C3 steps).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_c3prof}
mkdir -p $O
cd $R
timeout -k 10 200 python3 scripts/diag/c3_probe.py 10 > $O/c3_probe.log 2>&1 || { tail -20 $O/c3_probe.log; exit 1; }
cat $O/c3_probe.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 --output-format csv -- python3 $R/scripts/diag/c3_probe.py 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp $f $O/kernel_stats.csv
cut -d, -f1-4 $O/kernel_stats.csv | head -25
