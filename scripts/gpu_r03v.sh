set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03v; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo tests failed; grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -30; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp
for grp in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$grp -o run -- python3 $R/bench.py --kernel-only --steps 1 --warmup 0 > $OUT/pmc_$grp.log 2>&1 || { echo "pmc $grp failed"; tail -5 $OUT/pmc_$grp.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $OUT $OUT/pmc.json | grep -i "ops_compact\|classify\|walk<16\|fill<16"
for m in 0 1 2; do
CRISPR_NW_DEBUG_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/m$m -o k --output-format csv -- python3 $R/bench.py --kernel-only --steps 5 --warmup 1 > $OUT/m$m.log 2>&1 || { tail -20 $OUT/m$m.log; exit 1; }
echo "mode $m"; grep -h "nw_align_kernel\|ops_compact" $OUT/m$m/k_kernel_stats.csv | cut -c1-110
done
cd $R
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_EARLY_RUNS=0" 20 > $OUT/ab_early.log 2>&1 || { tail -20 $OUT/ab_early.log; exit 1; }
tail -2 $OUT/ab_early.log
