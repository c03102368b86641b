set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03y; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIRECT_OUT=0" 24 > $OUT/ab1.log 2>&1 || { tail -20 $OUT/ab1.log; exit 1; }
tail -2 $OUT/ab1.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIRECT_OUT=0" 6 pooled > $OUT/ab2.log 2>&1 || { tail -20 $OUT/ab2.log; exit 1; }
tail -2 $OUT/ab2.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIRECT_OUT=0" 8 c3 > $OUT/ab3.log 2>&1 || { tail -20 $OUT/ab3.log; exit 1; }
tail -2 $OUT/ab3.log
