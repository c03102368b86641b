#!/bin/bash
# Kernel + copy timeline of one pooled (C5) call: gpu_pooled_trace.sh [amplicons] [reads per amplicon]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/trace_pool -o run --output-format csv -- python3 $R/scripts/diag/pooled_call.py ${1:-96} ${2:-100000} > $R/gpurun_out/trace_pool.log 2>&1 || { tail -20 $R/gpurun_out/trace_pool.log; exit 1; }
cat $R/gpurun_out/trace_pool.log
python3 $R/scripts/diag/call_timeline.py $R/gpurun_out/trace_pool > $R/gpurun_out/timeline_pool.txt && tail -3 $R/gpurun_out/timeline_pool.txt
