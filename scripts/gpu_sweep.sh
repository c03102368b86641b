#!/bin/bash
# bench.py under a list of env settings (one line each: "VAR=v VAR2=w"); prints value + ms/step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
while read -r envs; do
  [ -z "$envs" ] && continue
  env $envs timeout -k 10 200 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-quant > $R/gpurun_out/sweep.log 2>&1 || { echo "FAIL $envs"; tail -5 $R/gpurun_out/sweep.log; exit 1; }
  echo "$envs :: $(grep '"metric"' $R/gpurun_out/sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M/s", round(d["ms_per_step"],3), "ms")')"
done < ${1:-/dev/stdin}
