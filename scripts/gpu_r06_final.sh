#!/bin/bash
# Round-6 measurement of HEAD in one lease: PMC passes (resident pass, call_pcie calls, quantification;
# scripts/gpu_pmc_call.sh), their summaries installed where bench.py reads them (profiles/r06_pmc on
# the box; commit the copies merged back under gpurun_out/pmc_<tag>/), then scripts/gpu_check.sh
# (GPU tests, smoke, the bench line, rocprofv3 kernel and call stats).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06_final}
cd $R
bash scripts/gpu_pmc_call.sh $TAG > /dev/null 2>&1 || { echo "PMC failed"; tail -20 gpurun_out/pmc_$TAG/*.log 2>/dev/null | tail -30; exit 1; }
mkdir -p profiles/r06_pmc
cp gpurun_out/pmc_$TAG/summary_*.json gpurun_out/pmc_$TAG/summary_*.txt profiles/r06_pmc/
echo "pmc ok"; tail -14 gpurun_out/pmc_$TAG/summary_resident.txt | cut -c1-200
bash scripts/gpu_check.sh $TAG
