#!/bin/bash
# Diagnostic: kernel time with later phases cut off (CRISPR_NW_DEBUG_MODE: 1 = fill + start cell only,
# 2 = + walk, 0 = full).  Optional first arg: extra env for all runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 0 1 2; do
  env CRISPR_NW_DEBUG_MODE=$m $1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/phase_$m.json 2>/dev/null || { echo FAIL $m; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/phase_$m.json'));r=d['roofline'];print('mode $m kernel_ms',round(r['kernel_ms_avg'],3), r.get('kernel_ms_split'))"
done
