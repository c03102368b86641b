#!/bin/bash
# bench headline vs CRISPR_NW_CHUNK (reads per pipeline chunk)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for c in ${CHUNKS:-131072 262144 393216 524288}; do
  CRISPR_NW_CHUNK=$c timeout -k 10 300 python bench.py --no-cpu --no-quant --no-legs --no-check > gpurun_out/sweep_$c.json 2> gpurun_out/sweep_$c.err || { echo FAIL $c; tail -5 gpurun_out/sweep_$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/sweep_$c.json')); print($c, round(d['value']/1e6,1), round(d['ms_per_step'],3), 'text', round(d['text_input']['value']/1e6,1), 'h2d', round(d['pcie']['h2d_ms'],3), 'comp', round(d['pcie']['compute_ms_in_call'],3), 'kernel', round(d['kernel_rate']['kernel_ms'],3))"
done
