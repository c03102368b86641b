#!/bin/bash
# Bench under several CRISPR_NW_* settings (one line each) after the GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for cfg in "${@:-default}"; do
  env $( [ "$cfg" = default ] || echo $cfg ) timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/sweep.json 2>gpurun_out/sweep.err || { echo BENCH_FAIL $cfg; tail -5 gpurun_out/sweep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sweep.json'));g=d['config']['kernel_geometry'];print('$cfg', round(d['value']/1e6,2),'Mreads/s', round(d['roofline']['kernel_ms_avg'],2),'ms', g)"
done
