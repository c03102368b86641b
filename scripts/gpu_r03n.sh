set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03n; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 10 c3 > $OUT/ab_c3_diag.log 2>&1 || { tail -20 $OUT/ab_c3_diag.log; exit 1; }
tail -2 $OUT/ab_c3_diag.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=0" 16 > $OUT/ab_c2_diag.log 2>&1 || { tail -20 $OUT/ab_c2_diag.log; exit 1; }
tail -2 $OUT/ab_c2_diag.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kprof -o kern --output-format csv -- python3 $R/bench.py --kernel-only --steps 10 --warmup 3 > $OUT/kprof.log 2>&1 || { tail -20 $OUT/kprof.log; exit 1; }
grep -h "^{" $OUT/kprof.log | cut -c1-400
