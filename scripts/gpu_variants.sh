#!/bin/bash
# Bench variants (headline + kernel pass only): gpu_variants.sh TAG "name:VAR=v,VAR=v" ...
# Optional GPU tests first: PYTEST_K="expr" runs pytest -m gpu -k expr.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=$1; shift
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" \
    > gpurun_out/vt_$TAG.log 2>&1 || { echo TESTS_FAIL; tail -60 gpurun_out/vt_$TAG.log; exit 1; }
  tail -2 gpurun_out/vt_$TAG.log
fi
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  [ "$envs" = "$spec" ] && envs=""
  ( IFS=','; for kv in $envs; do export "$kv"; done
    timeout -k 10 300 python bench.py --no-cpu --no-quant --no-legs --steps 10 > gpurun_out/v_${TAG}_$name.json 2> gpurun_out/v_${TAG}_$name.err ) \
    || { echo "FAIL $name"; tail -20 gpurun_out/v_${TAG}_$name.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/v_${TAG}_$name.json')); k=d['kernel_rate']
print('$name', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms; kernel', round(k['kernel_ms'],3), {a: round(b,3) for a,b in k['phases_ms'].items()}, k['path_counts'], 'mism', d.get('sample_check',{}).get('sample_mismatches'))"
done
