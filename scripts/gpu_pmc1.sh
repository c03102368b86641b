#!/bin/bash
# One PMC pass (VALU/SALU/LDS instruction counts, waves) of the default bench command
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
mkdir -p $R/gpurun_out/pmc1_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc1_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-quant > $R/gpurun_out/pmc1_$TAG/p.log 2>&1 || { echo PMC_FAIL; tail -5 $R/gpurun_out/pmc1_$TAG/p.log; exit 1; }
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc1_$TAG $R/gpurun_out/pmc1_$TAG/summary.json > /dev/null
python3 - $R/gpurun_out/pmc1_$TAG/summary.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    g=v.get("GRBM_GUI_ACTIVE",0)/8
    print(k[:40], "waves",v.get("SQ_WAVES"), "valu %.3g"%v.get("SQ_INSTS_VALU",0), "salu %.3g"%v.get("SQ_INSTS_SALU",0), "lds %.3g"%v.get("SQ_INSTS_LDS",0), "busy %.2f"%(v.get("SQ_INSTS_VALU",0)*4/(1024*g) if g else 0))
PY
