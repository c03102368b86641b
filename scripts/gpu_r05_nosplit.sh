#!/bin/bash
# A/B: every chunk's tail on its own compute stream (no tail stream) -- C1, C2, C3 dual, C5.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_nosplit}
mkdir -p $O
cd $R
timeout -k 10 200 python3 scripts/diag/ab_call.py "" "CRISPR_NW_NOSPLIT=1" 8 c1 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
timeout -k 10 150 python3 scripts/diag/ab_call.py "" "CRISPR_NW_NOSPLIT=1" 20 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
timeout -k 10 200 python3 scripts/diag/ab_call.py "" "CRISPR_NW_NOSPLIT=1" 8 dualonly >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
timeout -k 10 200 python3 scripts/diag/ab_call.py "" "CRISPR_NW_NOSPLIT=1" 6 pooled >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
