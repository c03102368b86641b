#!/bin/bash
# A/B: the lane walk + stop summary in the pipelined calls' chunks (C2 call, C3 dual call, C1, C5).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_lanecall}
mkdir -p $O
cd $R
timeout -k 10 150 python3 scripts/diag/ab_call.py "" "CRISPR_NW_LANECALL=1" 30 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
timeout -k 10 200 python3 scripts/diag/ab_call.py "" "CRISPR_NW_LANECALL=1" 10 dualonly >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
timeout -k 10 200 python3 scripts/diag/ab_call.py "" "CRISPR_NW_LANECALL=1" 8 c1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
timeout -k 10 200 python3 scripts/diag/ab_call.py "" "CRISPR_NW_LANECALL=1" 8 pooled >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
