set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03o; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 16 > $OUT/ab_c2_diag.log 2>&1 || { tail -20 $OUT/ab_c2_diag.log; exit 1; }
tail -2 $OUT/ab_c2_diag.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_MERGE=0" 16 > $OUT/ab_c2_merge.log 2>&1 || { tail -20 $OUT/ab_c2_merge.log; exit 1; }
tail -2 $OUT/ab_c2_merge.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 8 c3 > $OUT/ab_c3_diag.log 2>&1 || { tail -20 $OUT/ab_c3_diag.log; exit 1; }
tail -2 $OUT/ab_c3_diag.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 5 pooled > $OUT/ab_pooled_diag.log 2>&1 || { tail -20 $OUT/ab_pooled_diag.log; exit 1; }
tail -2 $OUT/ab_pooled_diag.log
timeout -k 10 200 python bench.py --kernel-only --steps 10 --warmup 3 > $OUT/kernel_only.json 2> $OUT/kernel_only.err || { tail -20 $OUT/kernel_only.err; exit 1; }
cut -c1-600 $OUT/kernel_only.json
