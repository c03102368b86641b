set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; tail -50 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python scripts/diag/ab_call.py "CRISPR_NW_PRIO=1" "CRISPR_NW_PRIO=0" 30 > $OUT/ab_prio_c2.log 2>&1 || { tail -20 $OUT/ab_prio_c2.log; exit 1; }
tail -4 $OUT/ab_prio_c2.log
timeout -k 10 200 python scripts/diag/ab_call.py "CRISPR_NW_PRIO=1" "CRISPR_NW_PRIO=0" 8 pooled > $OUT/ab_prio_c5.log 2>&1 || { tail -20 $OUT/ab_prio_c5.log; exit 1; }
tail -4 $OUT/ab_prio_c5.log
timeout -k 10 300 python scripts/diag/pooled_probe2.py c2:10 pooled:8 c4:4 pooled:8 c2:10 c4:4 c2:10 pooled:4 > $OUT/probe2.log 2>&1 || { tail -20 $OUT/probe2.log; exit 1; }
cat $OUT/probe2.log
