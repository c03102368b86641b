set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03q; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 16 > $OUT/ab1.log 2>&1 || { tail -20 $OUT/ab1.log; exit 1; }
tail -2 $OUT/ab1.log
timeout -k 10 300 python scripts/diag/ab_call.py "CRISPR_NW_DIAG_TAIL=3" "CRISPR_NW_DIAG_TAIL=1" 16 > $OUT/ab2.log 2>&1 || { tail -20 $OUT/ab2.log; exit 1; }
tail -2 $OUT/ab2.log
timeout -k 10 300 python scripts/diag/ab_call.py "CRISPR_NW_DIAG_TAIL=4" "CRISPR_NW_DIAG_TAIL=0" 16 > $OUT/ab3.log 2>&1 || { tail -20 $OUT/ab3.log; exit 1; }
tail -2 $OUT/ab3.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 5 c4 > $OUT/ab4.log 2>&1 || { tail -20 $OUT/ab4.log; exit 1; }
tail -2 $OUT/ab4.log
