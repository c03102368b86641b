#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CRISPR_NW_CHUNK=${1:-262144} timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/trace_call -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-quant --no-legs --no-check --skip-kernel-pass > $R/gpurun_out/trace_call.log 2>&1 || { tail -20 $R/gpurun_out/trace_call.log; exit 1; }
python3 $R/scripts/diag/call_timeline.py $R/gpurun_out/trace_call > $R/gpurun_out/timeline.txt && tail -160 $R/gpurun_out/timeline.txt
