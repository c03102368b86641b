#!/bin/bash
# A/B of the chunk-end events without timestamps: libcrispr_nw_r5prev.so (the parent commit's build) against
# this build on the C2, pooled (C5) and dual (C3) calls, libraries alternated; then the GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_events2}
mkdir -p $O
cd $R
for r in 1 2; do
  for l in libcrispr_nw_r5prev.so libcrispr_nw.so; do
    CRISPR_NW_LIB=$l timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 15 > $O/c2_$l.log 2>&1 || { tail -20 $O/c2_$l.log; exit 1; }
    echo "$l C2 $(grep '^A ' $O/c2_$l.log)"
    CRISPR_NW_LIB=$l timeout -k 10 300 python3 scripts/diag/ab_call.py "" "" 6 pooled > $O/c5_$l.log 2>&1 || { tail -20 $O/c5_$l.log; exit 1; }
    echo "$l C5 $(grep '^A ' $O/c5_$l.log)"
    CRISPR_NW_LIB=$l timeout -k 10 200 python3 scripts/diag/ab_call.py "" "" 10 dualonly > $O/c3_$l.log 2>&1 || { tail -20 $O/c3_$l.log; exit 1; }
    echo "$l C3 $(grep '^A ' $O/c3_$l.log)"
  done
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
