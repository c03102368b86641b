#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for sets in 1 2 3; do for c in 131072 262144; do
  CRISPR_NW_SETS=$sets CRISPR_NW_CHUNK=$c timeout -k 10 300 python bench.py --no-cpu --no-quant --no-legs --no-check > gpurun_out/ss_${sets}_${c}.json 2> gpurun_out/ss.err || { echo FAIL; tail -5 gpurun_out/ss.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ss_${sets}_${c}.json')); print('sets', $sets, 'chunk', $c, round(d['value']/1e6,1), round(d['ms_per_step'],3), 'text', round(d['text_input']['value']/1e6,1))"
done; done
