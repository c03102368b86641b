set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03s; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
CRISPR_NW_HOST_TIMING=1 timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 6 > $OUT/ht.log 2>&1 || { tail -20 $OUT/ht.log; exit 1; }
grep -v "^nw host\|^  chunk" $OUT/ht.log | tail -2; grep -B8 "^nw host" $OUT/ht.log | tail -36
