#!/bin/bash
# Timeline of the headline call: rocprofv3 kernel + memory-copy trace of a short bench run
# (call_timeline.py), then the call's host phases under CRISPR_NW_HOST_TIMING=1.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/trace_call -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-quant --no-legs --no-multi --no-check --skip-kernel-pass > $R/gpurun_out/trace_call.log 2>&1 || { tail -20 $R/gpurun_out/trace_call.log; exit 1; }
python3 $R/scripts/diag/call_timeline.py $R/gpurun_out/trace_call > $R/gpurun_out/timeline.txt && tail -40 $R/gpurun_out/timeline.txt
cd $R && CRISPR_NW_HOST_TIMING=1 timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 4 > gpurun_out/host_timing.log 2>&1 || { tail -20 gpurun_out/host_timing.log; exit 1; }
grep -v "^nw host" gpurun_out/host_timing.log | tail -3; grep "^nw host" gpurun_out/host_timing.log | tail -6
