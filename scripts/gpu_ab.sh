#!/bin/bash
# A/B of library variants: GPU tests on the default build, then one bench line per
# CRISPR_NW_LIB variant (arguments = extra .so names under crispresso_amd/lib).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for lib in libcrispr_nw.so "$@"; do
  for env in "" ${AB_ENVS:-}; do
    env CRISPR_NW_LIB=$lib $env timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo BENCH_FAIL $lib; tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$lib $env', round(d['value']/1e6,2),'Mreads/s', round(r['kernel_ms_avg'],2),'ms', {k: round(v,2) for k,v in r['kernel_ms_split'].items()}, d['config']['kernel_geometry'])"
  done
done
