set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03ab; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k -o k --output-format csv -- python3 $R/bench.py --kernel-only --steps 10 --warmup 3 > $OUT/k.log 2>&1 || { tail -20 $OUT/k.log; exit 1; }
grep -h "walk<16>\|ops_compact\|classify\|walk<32>" $OUT/k/k_kernel_stats.csv | awk -F',' '{print $1, $4}' | cut -c1-100
grep -h '^{' $OUT/k.log | cut -c1-200
cd $R
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_DIAGPASS=1" 5 c4 > $OUT/ab_c4.log 2>&1 || { tail -20 $OUT/ab_c4.log; exit 1; }
tail -2 $OUT/ab_c4.log
