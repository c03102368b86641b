set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03p; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 6 c4 > $OUT/ab_c4_diag.log 2>&1 || { tail -20 $OUT/ab_c4_diag.log; exit 1; }
tail -2 $OUT/ab_c4_diag.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 16 > $OUT/ab_c2_diag.log 2>&1 || { tail -20 $OUT/ab_c2_diag.log; exit 1; }
tail -2 $OUT/ab_c2_diag.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 6 pooled > $OUT/ab_pooled_diag.log 2>&1 || { tail -20 $OUT/ab_pooled_diag.log; exit 1; }
tail -2 $OUT/ab_pooled_diag.log
