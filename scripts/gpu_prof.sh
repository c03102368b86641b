#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command (no PMC): gpurun_out/prof_<tag>/
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
EXTRA=${2:-}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-quant $EXTRA > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
f=$(find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
head -12 "$f"
grep '"metric"' $R/gpurun_out/prof_$TAG.log | tail -c 400
