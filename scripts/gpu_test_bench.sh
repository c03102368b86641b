#!/bin/bash
# GPU parity tests, then the default bench line (no CPU baseline leg).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
