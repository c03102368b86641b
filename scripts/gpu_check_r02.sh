#!/bin/bash
# GPU tests (one process), smoke, then the default bench line.  Usage: gpu_check_r02.sh TAG [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
K=${2:-}
cd $R
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG="-k $K"; else KARG=""; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $KARG > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAIL; tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; cat gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
