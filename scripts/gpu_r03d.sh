set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python scripts/diag/ab_call.py "CRISPR_NW_DIAGPASS=1" "CRISPR_NW_DIAGPASS=0" 20 > $OUT/ab_diag_c2.log 2>&1 || { tail -20 $OUT/ab_diag_c2.log; exit 1; }
tail -4 $OUT/ab_diag_c2.log
timeout -k 10 200 python scripts/diag/ab_call.py "CRISPR_NW_PRIO=1" "CRISPR_NW_PRIO=0" 20 > $OUT/ab_prio_c2.log 2>&1 || { tail -20 $OUT/ab_prio_c2.log; exit 1; }
tail -4 $OUT/ab_prio_c2.log
timeout -k 10 200 python bench.py --kernel-only --steps 10 --warmup 3 > $OUT/kernel_only.json 2> $OUT/kernel_only.err || { tail -20 $OUT/kernel_only.err; exit 1; }
cat $OUT/kernel_only.json
CRISPR_NW_DIAGPASS=0 timeout -k 10 200 python bench.py --kernel-only --steps 10 --warmup 3 > $OUT/kernel_only_nodiag.json 2>> $OUT/kernel_only.err || { tail -20 $OUT/kernel_only.err; exit 1; }
cat $OUT/kernel_only_nodiag.json
