set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03z; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
CRISPR_NW_EXACT=multi timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k -o k --output-format csv -- python3 $R/bench.py --kernel-only --steps 5 --warmup 1 > $OUT/k.log 2>&1 || { tail -20 $OUT/k.log; exit 1; }
grep -h "exact\|nw_align_kernel" $OUT/k/k_kernel_stats.csv | cut -c1-120
cd $R
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_EXACT=multi" 20 > $OUT/ab1.log 2>&1 || { tail -20 $OUT/ab1.log; exit 1; }
tail -2 $OUT/ab1.log
