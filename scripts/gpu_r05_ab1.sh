#!/bin/bash
# Round 5 call experiments: per-launch trace of the last chunks, then in-process A/Bs of the
# call's knobs; the lane quantification tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_ab1}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_quant.py > $O/quant_tests.log 2>&1 || { tail -30 $O/quant_tests.log; exit 1; }
tail -2 $O/quant_tests.log
CRISPR_NW_TRACE=3 CRISPR_NW_HOST_TIMING=1 timeout -k 10 120 python3 scripts/diag/ab_call.py "" "" 2 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
R1=65536,131072,262144,262144,196608,65536,16960
R2=65536,131072,262144,262144,196608,49152,24576,8768
for ab in "CRISPR_NW_L2SKIP=1" "CRISPR_NW_SPIN=1" "CRISPR_NW_NOSPLIT_LAST=1" "CRISPR_NW_NOSPLIT_LAST=2" "CRISPR_NW_RAMP=$R1" "CRISPR_NW_RAMP=$R2" "CRISPR_NW_L2SKIP=1,CRISPR_NW_SPIN=1,CRISPR_NW_NOSPLIT_LAST=2,CRISPR_NW_RAMP=$R2"; do
  timeout -k 10 120 python3 scripts/diag/ab_call.py "" "$ab" 25 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
cat $O/ab.log
grep "trace chunk" $O/trace.log | tail -40
