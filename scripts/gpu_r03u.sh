set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03u; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
for m in 0 1 2; do
CRISPR_NW_DEBUG_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/m$m -o k --output-format csv -- python3 $R/bench.py --kernel-only --steps 5 --warmup 1 > $OUT/m$m.log 2>&1 || { tail -20 $OUT/m$m.log; exit 1; }
echo "mode $m"; grep -h "nw_align_kernel" $OUT/m$m/k_kernel_stats.csv | cut -c1-120
done
