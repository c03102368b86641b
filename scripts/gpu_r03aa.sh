set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r03aa; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests0.log 2>&1 || { echo tests failed; tail -30 $OUT/tests0.log; exit 1; }
CRISPR_NW_UPLOAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests1.log 2>&1 || { echo tests failed; tail -30 $OUT/tests1.log; exit 1; }
tail -1 $OUT/tests1.log
timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_UPLOAD=1" 24 > $OUT/ab1.log 2>&1 || { tail -20 $OUT/ab1.log; exit 1; }
tail -2 $OUT/ab1.log
CRISPR_NW_HOST_TIMING=1 timeout -k 10 300 python scripts/diag/ab_call.py "" "CRISPR_NW_UPLOAD=1" 3 > $OUT/ht.log 2>&1 || { tail -20 $OUT/ht.log; exit 1; }
grep -B8 "^nw host" $OUT/ht.log | tail -18
