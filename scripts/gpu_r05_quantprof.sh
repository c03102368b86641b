#!/bin/bash
# The quantification leg's kernels timed (rocprofv3 kernel stats of bench.py --quant-only).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_quantprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o q --output-format csv -- python3 $R/bench.py --quant-only --steps 10 --warmup 2 --no-cpu > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep '"metric"' $O/prof.log | cut -c1-300
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp $f $O/kernel_stats.csv
cut -d, -f1-4 $O/kernel_stats.csv | head -12
