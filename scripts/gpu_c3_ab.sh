#!/bin/bash
# C3 dual-alignment leg (and the rest of the bench line) under two env settings, alternating.
# Usage: gpu_c3_ab.sh "A-env" "B-env"
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for r in 1 2; do
  for spec in "$1" "$2"; do
    env $spec timeout -k 10 200 python bench.py --no-cpu --no-check --no-quant > gpurun_out/c3ab.json 2> gpurun_out/c3ab.err || { echo BENCH_FAIL; tail -5 gpurun_out/c3ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/c3ab.json'));print('[$spec]', 'C2', round(d['ms_per_step'],3), 'C3', round(d['dual_alignment']['ms_per_step'],3), 'C5', round(d['pooled']['ms_per_step'],3), d['kernel_rate']['path_counts'])"
  done
done
