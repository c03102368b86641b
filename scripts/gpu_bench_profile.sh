#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_r01.err; exit 1; }
cat gpurun_out/bench_r01.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r01 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof_r01.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof_r01.log; exit 1; }
find $R/gpurun_out/prof_r01 -name "*stats*" | head
